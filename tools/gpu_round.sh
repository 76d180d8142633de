#!/bin/bash
# One GPU call: smoke, GPU parity tests, bench (each step time-limited; stop at first failure).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m4 -E "gfx950|Marketing Name" > gpurun_out/rocminfo.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
[ -n "${NO_BENCH}" ] && exit 0
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
