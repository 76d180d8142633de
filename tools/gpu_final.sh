#!/bin/bash
# End-of-session evidence: the default bench line and every BASELINE config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
tail -c 300 gpurun_out/bench.json
timeout -k 10 400 python3 tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { tail -20 gpurun_out/configs.err; exit 1; }
cat gpurun_out/configs.jsonl
