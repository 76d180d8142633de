#!/bin/bash
# Phase stamps and per-evaluation durations of the in-tree build for several speculation caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cap in ${CAPS:-0 2 4}; do
  FMPNP_SPEC_CAP=$cap SPEC=1 timeout -k 10 120 python3 tools/diag_phases.py 128 > gpurun_out/phases_cap$cap.log 2>&1 || exit 1
  FMPNP_DBG=4 FMPNP_SPEC_CAP=$cap timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_cap$cap.log 2>&1 || exit 1
done
