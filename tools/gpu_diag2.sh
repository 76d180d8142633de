#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for a in "128 0" "128 1" "128 2" "128 8" "1 0" "1 8" "256 0"; do
timeout -k 10 300 python tools/diag_phases.py $a 2>&1 | grep -v amdgpu.ids || exit 1
done
