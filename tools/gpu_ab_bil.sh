#!/bin/bash
# GPU bilinear tests, then an interleaved A/B of the bilinear memo leg (B=128) against ab_old/head.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_bilinear.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bil.log 2>&1 || { tail -40 gpurun_out/pytest_bil.log; exit 1; }
tail -1 gpurun_out/pytest_bil.log
for i in 1 2 3; do
  for arm in "FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so" "X=1"; do
    timeout -k 10 200 env $arm python3 bench.py --legs none --sampling bilinear --steps ${STEPS:-400} --warmup 5 > gpurun_out/abb.json 2> gpurun_out/abb.err || { tail gpurun_out/abb.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/abb.json').read().strip().splitlines()[-1])
print('[$arm] ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'])"
  done
done
