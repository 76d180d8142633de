#!/bin/bash
# Copy the summaries of tools/gpu_profile_all.sh from gpurun_out/prof/ into profiles/ as round RNN.
#   tools/collect_profiles.sh r04
R=${1:?round tag, e.g. r04}
cd "$(dirname "$0")/.." || exit 1
P=gpurun_out/prof
for d in "$P"/b*/; do
  t=$(basename "$d")
  [ -f "$d/summary.json" ] && cp "$d/summary.json" "profiles/${R}_pmc_$t.json"
  [ -f "$d/kernel_stats.csv" ] && cp "$d/kernel_stats.csv" "profiles/${R}_rocprof_kernel_stats_$t.csv"
done
[ -f "$P/sq/summary.txt" ] && cp "$P/sq/summary.txt" "profiles/${R}_sq_b128.txt"
[ -f "$P/pipeline/summary.json" ] && cp "$P/pipeline/summary.json" "profiles/${R}_pmc_pipeline.json"
[ -f "$P/pipeline_w5/summary.json" ] && cp "$P/pipeline_w5/summary.json" "profiles/${R}_pmc_pipeline_w5.json"
[ -f "$P/pipeline_robotcar/summary.json" ] && cp "$P/pipeline_robotcar/summary.json" "profiles/${R}_pmc_pipeline_robotcar.json"
for d in "$P"/facade_*/; do
  t=$(basename "$d")
  [ -f "$d/summary.json" ] && cp "$d/summary.json" "profiles/${R}_pmc_$t.json"
  [ -f "$d/kernel_stats.csv" ] && cp "$d/kernel_stats.csv" "profiles/${R}_rocprof_kernel_stats_$t.csv"
done
for n in 866 295; do
  [ -f "$P/pyramid_n$n/summary.json" ] && cp "$P/pyramid_n$n/summary.json" "profiles/${R}_pmc_pyramid_n$n.json"
done
if [ -f "$P/tatd/run_counter_collection.csv" ]; then
  python3 - "$P/tatd/run_counter_collection.csv" > "profiles/${R}_tatd_b128.txt" <<'PY'
import csv, sys, collections
tot = collections.defaultdict(float); n = collections.defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    if "lm_kernel" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print("B=128 headline LM kernel (bench.py --legs none --steps 5), per dispatch, summed over instances:")
for k in sorted(tot):
    print(f"  {k:18s} {tot[k] / len(n[k]):14.0f}  ({len(n[k])} dispatches)")
g = tot["GRBM_GUI_ACTIVE"] / len(n["GRBM_GUI_ACTIVE"]) / 8   # GRBM_GUI_ACTIVE sums the 8 XCDs
for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum"):
    if k in tot:
        per_cu = tot[k] / len(n[k]) / 128   # the 128 CUs that hold a workgroup
        print(f"  {k}: {per_cu:.0f} busy cycles per active CU = {per_cu / g:.1%} of the kernel's {g:.0f} cycles")
PY
fi
ls -la profiles | grep "${R}_" | wc -l
