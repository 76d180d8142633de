#!/bin/bash
# pack kernel HBM traffic: rocprofv3 FETCH_SIZE and WRITE_SIZE passes (kernel trace only,
# one counter group per pass) over tools/bench_pack.py at the cfg2 shape
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/pack_pmc"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$REPO/tools/bench_pack.py" 256 240 320 > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "$REPO/tools/bench_pack.py" 256 240 320 > "$OUT/fetch.log" 2>&1 || { tail -20 "$OUT/fetch.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "$REPO/tools/bench_pack.py" 256 240 320 > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics
out = sys.argv[1]
def rows(kind):
    f = glob.glob(f"{out}/{kind}/**/*counter_collection.csv", recursive=True)[0]
    return [r for r in csv.DictReader(open(f)) if "sobel_pack" in r["Kernel_Name"]]
fe = [float(r["Counter_Value"]) for r in rows("fetch")]
wr = [float(r["Counter_Value"]) for r in rows("write")]
st = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)[0]
avg = [float(r["AverageNs"]) for r in csv.DictReader(open(st)) if "sobel_pack" in r["Name"]][0]
print("sobel_pack dispatches", len(fe), "avg ns", avg)
print("FETCH_SIZE KiB median", statistics.median(fe), "-> x2 bytes", 2 * 1024 * statistics.median(fe))
print("WRITE_SIZE KiB median", statistics.median(wr), "-> bytes", 1024 * statistics.median(wr))
print("algorithmic: read", 4 * 256 * 240 * 320, "write", 12 * 256 * 240 * 320)
PY
