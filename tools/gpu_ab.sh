#!/bin/bash
# A/B of two library builds on the headline (B=128) and the single query, interleaved:
# A = ab_old/ (FMPNP_LIB_PATH), B = the in-tree build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
run() {
  timeout -k 10 200 env $1 python3 bench.py --legs single --steps ${STEPS:-4000} --warmup 20 ${EXTRA} > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('$2 ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'], 'single', d['single_query']['ms_per_refinement'])"
}
for i in 1 2 3; do
  run "FMPNP_LIB_PATH=$PWD/ab_old/featuremetric-pnp_amd/fmpnp/lib/libfmpnp.so" A || exit 1
  run "X=1" B || exit 1
done
