#!/bin/bash
# Phase stamps of the LM kernel (tools/diag_phases.py): bilinear memo at B=128, nearest at B=128 and B=1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
SPEC=0 SAMPLING=bilinear timeout -k 10 120 python3 tools/diag_phases.py ${B:-128} > gpurun_out/phases_bil.log 2>&1 || exit 1
[ -n "$BIL_ONLY" ] && exit 0
SPEC=0 timeout -k 10 120 python3 tools/diag_phases.py 128 > gpurun_out/phases_nn128.log 2>&1 && SPEC=0 timeout -k 10 120 python3 tools/diag_phases.py 1 > gpurun_out/phases_nn1.log 2>&1
