#!/bin/bash
# rocprofv3 kernel trace + stats of the bench, then PMC passes (FETCH_SIZE and WRITE_SIZE
# separately, kernel trace only) and a summary (tools/pmc_summary.py) in gpurun_out/prof.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BATCH="${BATCH:-128}"
ARGS="${BENCH_ARGS:---steps 5 --warmup 1 --no-extras --no-nomemo --no-bilinear --no-layout-f} --batch $BATCH"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$REPO/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { echo "trace failed"; tail -20 "$OUT/trace.err"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_write.err" || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 1; }
python3 "$REPO/tools/pmc_summary.py" "$OUT" "$BATCH" "$OUT/summary.json"
cat "$OUT/trace_bench.json"
