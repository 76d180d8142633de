#!/bin/bash
# Bilinear cell memo on the GPU: parity tests, then bench lines of the memo and direct forms.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$REPO"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_bilinear.py -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/bil_tests.log 2>&1 || { tail -40 gpurun_out/bil_tests.log; exit 1; }
tail -3 gpurun_out/bil_tests.log
timeout -k 10 200 python3 bench.py --legs none --steps 20 --warmup 2 --sampling bilinear > gpurun_out/bil_memo.json 2> gpurun_out/bil_memo.err || { tail gpurun_out/bil_memo.err; exit 1; }
timeout -k 10 200 python3 bench.py --legs none --steps 5 --warmup 1 --sampling bilinear --no-memo > gpurun_out/bil_direct.json 2> gpurun_out/bil_direct.err || { tail gpurun_out/bil_direct.err; exit 1; }
python3 - <<'PY'
import json
for f in ("gpurun_out/bil_memo.json", "gpurun_out/bil_direct.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["value"], d["config"]["launch"], d["roofline"]["texel_gathers_per_point_eval"])
PY
