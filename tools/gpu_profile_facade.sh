#!/bin/bash
# rocprofv3 of the reference consumer's per-call path (tools/facade_call.py): per shape one kernel-trace +
# stats run (24 timed calls + 2 warm-up) and separate FETCH_SIZE / WRITE_SIZE runs (4 + 2 calls), summarised
# by tools/pmc_facade_summary.py into gpurun_out/prof/facade_<shape>/summary.json.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/prof"
cd /tmp && export TMPDIR=/tmp
for s in ${SHAPES:-cfg2 robotcar_n295 robotcar_n866}; do
  D="$OUT/facade_$s"; mkdir -p "$D"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 "$REPO/tools/facade_call.py" $s --calls 24 > "$D/trace.json" 2> "$D/trace.err" || { echo "trace $s failed"; tail -5 "$D/trace.err"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 "$REPO/tools/facade_call.py" $s --calls 4 > /dev/null 2> "$D/fetch.err" || { echo "fetch $s failed"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 "$REPO/tools/facade_call.py" $s --calls 4 > /dev/null 2> "$D/write.err" || { echo "write $s failed"; exit 1; }
  python3 "$REPO/tools/pmc_facade_summary.py" "$D" $s 26 6 || exit 1
  find "$D/trace" -name "*kernel_stats.csv" -exec cp {} "$D/kernel_stats.csv" \;
  rm -rf "$D/trace" "$D/pmc_fetch" "$D/pmc_write"
done
