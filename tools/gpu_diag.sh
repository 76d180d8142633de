#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_batch.py > gpurun_out/diag.log 2>&1; rc=$?
cat gpurun_out/diag.log | grep -v amdgpu.ids
exit $rc
