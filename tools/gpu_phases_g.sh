#!/bin/bash
# Phase stamps of the LM kernel at B=128 for G = 1, 2, 4 workgroups per problem (8-wave build).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for g in 1 2 4; do
  SPEC=0 timeout -k 10 120 python3 tools/diag_phases.py ${B:-128} $g > gpurun_out/phases_g$g.log 2>&1 || exit 1
done
