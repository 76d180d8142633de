#!/bin/bash
# Per-evaluation diagnostics of the headline launch on the GPU box, with a stamps build
# (tools/build_ab.sh stamps -- -DFMPNP_STAMPS=1):
#   tools/gpu_diag.sh TAG [LIB]     -> gpurun_out/<TAG>_timeline_e<E>.txt, <TAG>_evals.txt
# env: EVALS (default "5 20 40"), B (128), INIT (easy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${1:-diag}
LIB=${2:-$PWD/ab_old/stamps/libfmpnp.so}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 FMPNP_LIB_PATH=$LIB
for e in ${EVALS:-5 20 40}; do
  timeout -k 10 120 python3 tools/diag_timeline.py ${B:-128} $e ${INIT:-easy} > gpurun_out/${TAG}_timeline_e$e.txt 2>&1 \
      || { tail -5 gpurun_out/${TAG}_timeline_e$e.txt; exit 1; }
  cat gpurun_out/${TAG}_timeline_e$e.txt
done
FMPNP_DBG=4 timeout -k 10 120 python3 tools/diag_evals.py ${B:-128} 0 ${INIT:-easy} > gpurun_out/${TAG}_evals.txt 2>&1 \
    || { tail -5 gpurun_out/${TAG}_evals.txt; exit 1; }
cat gpurun_out/${TAG}_evals.txt
