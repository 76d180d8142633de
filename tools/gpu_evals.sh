#!/bin/bash
# Per-evaluation durations (tools/diag_evals.py) at B=128 and B=1, easy and hard starts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export FMPNP_DBG=4
timeout -k 10 120 python3 tools/diag_evals.py 128 0 easy > gpurun_out/evals_b128_easy.log 2>&1 &&
timeout -k 10 120 python3 tools/diag_evals.py 1 0 easy > gpurun_out/evals_b1_easy.log 2>&1 &&
timeout -k 10 120 python3 tools/diag_evals.py 128 0 hard > gpurun_out/evals_b128_hard.log 2>&1 &&
timeout -k 10 120 python3 tools/diag_evals.py 128 2 easy > gpurun_out/evals_b128_g2.log 2>&1
