#!/bin/bash
# Headline B=128 under different builds: default (8 waves, G=1), wide (4 waves, one per SIMD) with G=1/2/4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run() {
  timeout -k 10 200 env $1 python3 bench.py --legs single --steps 3000 --warmup 20 $2 > gpurun_out/w.json 2> gpurun_out/w.err || { tail gpurun_out/w.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/w.json').read().strip().splitlines()[-1])
print('$1 $2', 'ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'], 'single', d['single_query']['ms_per_refinement'], d['config']['launch'], d['statuses'])"
}
run "X=1" "" && run "FMPNP_LM_WPS=1" "--wgs 2" && run "FMPNP_LM_WPS=1" "--wgs 1" && run "FMPNP_LM_WPS=1" "--wgs 4" && run "X=1" "--wgs 2" && run "FMPNP_LM_WPS=1" "--wgs 2 --batch 256"  && run "X=1" "--batch 256"
