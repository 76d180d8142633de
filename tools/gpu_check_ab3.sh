#!/bin/bash
# GPU tests of the in-tree build, then an interleaved A/B against ab_old/head and per-evaluation stamps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
FMPNP_DBG=4 timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_new.log 2>&1 && grep total gpurun_out/evals_new.log
ARMS="FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so;X=1" bash tools/gpu_ab_env.sh
