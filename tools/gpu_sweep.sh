#!/bin/bash
# phase-share sweep: SWEEP="B:G B:G ..." (G = 0 -> auto)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for bg in ${SWEEP:-128:0 128:4 128:8 256:0 1:0 1:16}; do
timeout -k 10 300 python tools/diag_phases.py ${bg%%:*} ${bg##*:} 2>&1 | grep -v amdgpu.ids || exit 1
done
