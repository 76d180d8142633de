#!/bin/bash
# GPU tests, then per-evaluation stamps for several caps and an interleaved A/B against ab_old/head.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cap in ${CAPS:-0 2 4}; do
  FMPNP_DBG=4 FMPNP_SPEC_CAP=$cap timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_cap$cap.log 2>&1 || exit 1
  echo "cap $cap: $(grep total gpurun_out/evals_cap$cap.log)"
done
ARMS="FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so;X=1;FMPNP_SPEC_CAP=2" bash tools/gpu_ab_env.sh
