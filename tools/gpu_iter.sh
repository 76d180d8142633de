#!/bin/bash
# iteration loop: GPU tests, phase diagnostics, short bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
bash tools/gpu_check.sh || exit 1
for a in ${DIAG_CASES:-"128 0" "1 0" "256 0"}; do :; done
timeout -k 10 300 python tools/diag_phases.py 128 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/diag_phases.py 1 0 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python tools/diag_phases.py 256 0 2>&1 | grep -v amdgpu.ids || exit 1
BENCH_ARGS="--steps 5 --warmup 1 --cpu-sample 0" bash tools/gpu_bench.sh
