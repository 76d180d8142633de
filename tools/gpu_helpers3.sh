#!/bin/bash
# GPU tests, smoke; batch sweep around the helpers' limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for B in 1 64 85 128; do
  for hv in 0 1; do
    FMPNP_HELPERS=$hv timeout -k 10 200 python3 bench.py --legs none --batch $B --steps 2000 --warmup 10 > gpurun_out/hb.json 2> gpurun_out/hb.err || { tail gpurun_out/hb.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/hb.json').read().strip().splitlines()[-1])
print('B=$B helpers=$hv ms_per_step', d['ms_per_step'], 'grid', d['config']['launch']['grid'])"
  done
done
