#!/bin/bash
# Per-evaluation durations of the speculation build (ab_old/spec): which waves speculate, caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_LIB_PATH=$PWD/ab_old/spec/libfmpnp.so FMPNP_DBG=4
for cfg in "4 4" "4 8" "4 64" "1 4" "0 4"; do
  set -- $cfg
  FMPNP_SPEC_W0=$1 FMPNP_SPEC_CAP=$2 timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_w$1_cap$2.log 2>&1 || exit 1
done
unset FMPNP_DBG
FMPNP_SPEC_W0=4 FMPNP_SPEC_CAP=8 SPEC=1 timeout -k 10 120 python3 tools/diag_phases.py 128 > gpurun_out/phases_w4_cap8.log 2>&1
