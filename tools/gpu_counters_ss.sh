#!/bin/bash
# SQ and TA/TD counters of the headline with the opt-in steady-state gather helpers (FMPNP_SS=1,
# VAR_GM_SS) for the comparison with the shipped speculation (profiles/r04_sq_b128.txt,
# r04_tatd_b128.txt): separate counter passes, kernel trace only (MI355X_MICROARCH.md).
#   -> gpurun_out/prof/ss/{sq.txt,tatd.txt}
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
D="$REPO/gpurun_out/prof/ss"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
export FMPNP_SS=1
ARGS="--legs none --steps 5 --warmup 1 --batch 128"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS" \
           "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d "$D/p$i" -o run -- python3 "$REPO/bench.py" $ARGS > "$D/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$D/p$i.log"; exit 1; }
done
python3 - "$D" > "$D/summary.txt" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(set); names = set()
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lm_kernel" in r["Kernel_Name"]:
            names.add(r["Kernel_Name"][:60])
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]].add(r["Dispatch_Id"])
print("kernel:", sorted(names))
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(1, len(n[k])):16.0f}  (per dispatch, {len(n[k])} dispatches)")
PY
cat "$D/summary.txt"
rm -rf "$D"/p1 "$D"/p2 "$D"/p3
