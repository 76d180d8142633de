#!/bin/bash
# Speculation build (ab_old/spec) with two workgroups per problem at B=128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_LIB_PATH=$PWD/ab_old/spec/libfmpnp.so
for cfg in "0 4" "1 4" "0 8"; do
  set -- $cfg
  FMPNP_DBG=4 FMPNP_SPEC_W0=$1 FMPNP_SPEC_CAP=$2 timeout -k 10 120 python3 tools/diag_evals.py 128 2 easy > gpurun_out/evals_g2_w$1_cap$2.log 2>&1 || exit 1
done
FMPNP_SPEC_W0=0 FMPNP_SPEC_CAP=4 SPEC=1 timeout -k 10 120 python3 tools/diag_phases.py 128 2 > gpurun_out/phases_g2_w0_cap4.log 2>&1
