#!/bin/bash
# Round evidence: GPU tests, rocprofv3 kernel stats + FETCH/WRITE_SIZE passes (B=128),
# then the default bench line (which reads the committed traffic summary).
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$REPO"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
BATCH=128 bash tools/gpu_profile.sh > gpurun_out/profile.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/profile.log; exit 1; }
cp gpurun_out/prof/summary.json profiles/pmc_traffic.json  # (on the box; copy it back from gpurun_out/prof/ locally)
cd "$REPO"
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
