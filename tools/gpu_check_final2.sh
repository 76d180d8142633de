#!/bin/bash
# GPU tests, every BASELINE config, and an interleaved A/B of the headline against ab_old/head.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { tail -20 gpurun_out/configs.err; exit 1; }
cut -c1-140 gpurun_out/configs.jsonl
ARMS="FMPNP_LIB_PATH=$PWD/ab_old/head/libfmpnp.so;X=1" bash tools/gpu_ab_env.sh
