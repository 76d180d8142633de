#!/bin/bash
# GPU tests, an interleaved A/B of the ratio-test leg (B=128, ratio 0.8) against ab_old/head, and
# the pipeline batch-shape sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2 3; do
  for arm in "FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so" "X=1"; do
    for init in easy hard; do
      timeout -k 10 200 env $arm python3 bench.py --legs none --ratio 0.8 --init $init --steps 2000 --warmup 10 > gpurun_out/abr.json 2> gpurun_out/abr.err || { tail gpurun_out/abr.err; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/abr.json').read().strip().splitlines()[-1])
print('[$arm] $init ms_per_step', d['ms_per_step'])"
    done
  done
done
bash tools/gpu_pipe_sweep.sh
