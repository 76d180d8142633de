#!/bin/bash
# pack kernel: parity tests + microbench (row-direction alternation on/off)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/ -x -q -m gpu -k "pack" --timeout 120 --timeout-method thread > gpurun_out/pytest_pack.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_pack.log; exit 1; }
tail -2 gpurun_out/pytest_pack.log
timeout -k 10 200 python -u tools/bench_pack.py ${PACK_SHAPES} || exit 1
FMPNP_PACK_ALT=0 timeout -k 10 200 python -u tools/bench_pack.py ${PACK_SHAPES}
