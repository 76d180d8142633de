#!/bin/bash
# Phase stamps of the speculation build (ab_old/spec) for per-wave caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_LIB_PATH=$PWD/ab_old/spec/libfmpnp.so
for cap in ${CAPS:-2 4}; do
  SPEC=1 FMPNP_SPEC_CAP=$cap timeout -k 10 120 python3 tools/diag_phases.py 128 > gpurun_out/phases_cap$cap.log 2>&1 || exit 1
done
