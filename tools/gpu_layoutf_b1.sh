#!/bin/bash
# Layout F single query / small batches: the planner's spread (G > 1) against one workgroup.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for B in 1 8; do
  for g in 0 1 2 4; do
    timeout -k 10 200 python3 bench.py --legs none --layout f --batch $B --wgs $g --steps 2000 --warmup 10 > gpurun_out/lf.json 2> gpurun_out/lf.err || { tail gpurun_out/lf.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/lf.json').read().strip().splitlines()[-1])
print('layout f B=$B wgs=$g ms_per_step', d['ms_per_step'], d['config']['launch'])"
  done
done
