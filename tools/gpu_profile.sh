#!/bin/bash
# rocprofv3 profiles of bench.py workloads on the GPU box.  For every workload: one kernel-trace
# + stats pass, then SEPARATE FETCH_SIZE and WRITE_SIZE passes (kernel trace only, as
# MI355X_MICROARCH.md prescribes), summarised by tools/pmc_summary.py into
# gpurun_out/prof/<tag>/summary.json (copy to profiles/rNN_pmc_<tag>.json) and
# gpurun_out/prof/<tag>/kernel_stats.csv (copy to profiles/rNN_rocprof_kernel_stats_<tag>.csv).
#   WORKLOADS="tag|bench flags" lines (tag = b<batch>_...); default: the headline.
#   SQ=1: also the SQ counters of the headline (two passes of <= 8 SQ counters).
#   TRACE_ARGS / PMC_ARGS: bench.py arguments of the trace / counter passes.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/prof"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
WORKLOADS="${WORKLOADS:-b128_easy|}"
TRACE_ARGS="${TRACE_ARGS:---legs none --steps 100 --warmup 3 --event-every 1}"
PMC_ARGS="${PMC_ARGS:---legs none --steps 5 --warmup 1}"
while IFS='|' read -r tag flags; do
  [ -z "$tag" ] && continue
  B=$(echo "$tag" | sed -E 's/^b([0-9]+)_.*/\1/')
  D="$OUT/$tag"; mkdir -p "$D"
  echo "[profile] $tag: $flags"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 "$REPO/bench.py" $TRACE_ARGS --batch $B $flags > "$D/bench.json" 2> "$D/trace.err" || { echo "trace $tag failed"; tail -20 "$D/trace.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 "$REPO/bench.py" $PMC_ARGS --batch $B $flags > /dev/null 2> "$D/pmc_fetch.err" || { echo "fetch $tag failed"; tail -20 "$D/pmc_fetch.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 "$REPO/bench.py" $PMC_ARGS --batch $B $flags > /dev/null 2> "$D/pmc_write.err" || { echo "write $tag failed"; tail -20 "$D/pmc_write.err"; exit 1; }
  python3 "$REPO/tools/pmc_summary.py" "$D" "$B" "$D/summary.json" auto "$tag" || exit 1
  find "$D/trace" -name "*kernel_stats.csv" -exec cp {} "$D/kernel_stats.csv" \;
  rm -rf "$D/trace" "$D/pmc_fetch" "$D/pmc_write"
done <<< "$WORKLOADS"
if [ -n "$SQ" ]; then
  D="$OUT/sq"; mkdir -p "$D"; i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$D/p$i" -o run -- python3 "$REPO/bench.py" $PMC_ARGS --batch 128 > "$D/p$i.log" 2>&1 || { echo "sq pass $i failed"; tail -5 "$D/p$i.log"; exit 1; }
  done
  python3 - "$D" > "$D/summary.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lm_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(1, len(n[k])):16.0f}  (per dispatch, {len(n[k])} dispatches)")
PY
  cat "$D/summary.txt"
  rm -rf "$D"/p1 "$D"/p2
fi
for f in "$OUT"/*/summary.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['tag'], d['kernel'], d['kernel_avg_ns'], d['hbm_bytes_per_launch'])" "$f"; done
