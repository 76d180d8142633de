#!/bin/bash
# Per-evaluation durations of the speculation build (ab_old/spec) for several per-wave caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_LIB_PATH=$PWD/ab_old/spec/libfmpnp.so FMPNP_DBG=4
for cap in ${CAPS:-0 2 4 6 64}; do
  FMPNP_SPEC_CAP=$cap timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_cap$cap.log 2>&1 || exit 1
done
unset FMPNP_LIB_PATH
timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_nospec.log 2>&1
