#!/bin/bash
# rocprofv3 kernel trace + stats, then PMC passes (FETCH_SIZE, WRITE_SIZE separately) of the bench.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="${BENCH_ARGS:---steps 5 --warmup 1 --no-extras}"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$REPO/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err" || { echo "trace failed"; tail -20 "$OUT/trace.err"; exit 1; }
echo "== stats"; find "$OUT/trace" -name "*kernel_stats.csv" -exec cat {} \;
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_fetch.err" || { echo "pmc fetch failed"; tail -20 "$OUT/pmc_fetch.err"; exit 1; }
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$REPO/bench.py" $ARGS > /dev/null 2> "$OUT/pmc_write.err" || { echo "pmc write failed"; tail -20 "$OUT/pmc_write.err"; exit 1; }
echo "== pmc files"; find "$OUT" -name "*.csv" | head -20
