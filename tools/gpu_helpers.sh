#!/bin/bash
# GPU tests, then single-query / small-batch timings with and without first-evaluation helpers.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for i in 1 2; do
  for hv in 0 1; do
    FMPNP_HELPERS=$hv timeout -k 10 300 python3 tools/bench_configs.py > gpurun_out/configs_h$hv.jsonl 2> gpurun_out/configs.err || { tail -20 gpurun_out/configs.err; exit 1; }
    echo "helpers=$hv"; cut -c1-120 gpurun_out/configs_h$hv.jsonl
  done
done
ARMS="FMPNP_HELPERS=0;FMPNP_HELPERS=1" bash tools/gpu_ab_env.sh
