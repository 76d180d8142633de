#!/bin/bash
# LM kernel iteration: GPU parity tests, phase stamps (B=128, B=1), short bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u tools/diag_phases.py 128 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 200 python -u tools/diag_phases.py 1 2>&1 | grep -v amdgpu.ids || exit 1
[ -n "${NO_BENCH}" ] && exit 0
timeout -k 10 300 python -u bench.py --cpu-sample 0 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.load(open("gpurun_out/bench.json"))
print("bench value", d["value"], "ms", d["ms_per_step"], "kernel_ms", d["roofline"]["avg_kernel_ms"], "no_memo", d.get("no_memo", {}).get("ms_per_launch"), "single", d.get("single_query", {}).get("ms_per_refinement"), "pack", d.get("pack", {}).get("ms"))
PY
