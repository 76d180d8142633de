#!/bin/bash
# Interleaved A/B of library builds / env settings on the headline (B=128) bench line.
# ARMS: ';'-separated env assignments per arm, e.g. "X=1;FMPNP_LIB_PATH=ab_old/spec/libfmpnp.so FMPNP_SPEC_CAP=4"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
IFS=';' read -ra arms <<< "$ARMS"
for i in 1 2 3; do
  k=0
  for arm in "${arms[@]}"; do
    timeout -k 10 200 env $arm python3 bench.py --legs single --steps ${STEPS:-4000} --warmup 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print('arm $k [$arm] ms_per_step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'], 'single', d['single_query']['ms_per_refinement'], 'spec', d['config']['speculative_gathers'])"
    k=$((k+1))
  done
done
