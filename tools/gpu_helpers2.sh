#!/bin/bash
# GPU tests; headline A/B against ab_old/head; batch sweep with and without first-evaluation helpers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
ARMS="FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so;X=1" bash tools/gpu_ab_env.sh || exit 1
for B in 1 8 32 64 85; do
  for hv in 0 1; do
    FMPNP_HELPERS=$hv timeout -k 10 200 python3 bench.py --legs none --batch $B --steps 2000 --warmup 10 > gpurun_out/hb.json 2> gpurun_out/hb.err || { tail gpurun_out/hb.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/hb.json').read().strip().splitlines()[-1])
print('B=$B helpers=$hv ms_per_step', d['ms_per_step'], 'grid', d['config']['launch']['grid'])"
  done
done
