#!/bin/bash
# rocprofv3 kernel stats of the streamed end-to-end pipeline (layout F): f-only pack,
# reference gather, LM launches, 8 batches x 128 queries
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/pipe_prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$REPO/tools/bench_pipeline.py" 8 128 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.log" | tail -1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "fmpnp" in r["Name"]:
        print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg", r["Percentage"], "%")
PY
