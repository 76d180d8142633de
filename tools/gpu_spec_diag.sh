#!/bin/bash
# Phase stamps and per-evaluation durations of the speculation build (ab_old/spec) at B=128.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_LIB_PATH=$PWD/ab_old/spec/libfmpnp.so
SPEC=1 timeout -k 10 120 python3 tools/diag_phases.py 128 > gpurun_out/phases_spec.log 2>&1 &&
FMPNP_DBG=4 timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_spec.log 2>&1
