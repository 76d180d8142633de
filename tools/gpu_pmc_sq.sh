#!/bin/bash
# SQ counters of the LM kernel (tools/diag_phases.py workload): instruction mix and wait states.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/pmc_sq"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="${B:-128}"; G="${G:-1}"
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" "$OUT/counters_list.txt" | sort -u > "$OUT/sq_names.txt" || true
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VALU_FMA_F64" "SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_EXP SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- python3 "$REPO/tools/diag_phases.py" $B $G > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
done
python3 - "$OUT" <<'PY'
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
