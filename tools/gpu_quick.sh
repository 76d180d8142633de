#!/bin/bash
# Headline timing only (plus single query): quick A/B of LM kernel changes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python3 bench.py --legs single --steps 4000 --warmup 20 > gpurun_out/quick$i.json 2> gpurun_out/quick.err || { tail gpurun_out/quick.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/quick$i.json').read().strip().splitlines()[-1])
print('B=128 ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'], 'value', d['value'], 'single', d['single_query']['ms_per_refinement'])"
done
