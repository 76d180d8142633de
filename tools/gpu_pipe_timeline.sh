#!/bin/bash
# Timeline of the streamed pipeline: per-dispatch kernel trace, then the span, the busy time
# of each kernel family and how much of the LM time overlaps pack/gather; plus a host profile.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/pipe_tl"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 "$REPO/tools/bench_pipeline.py" 4 128 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
k = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
k.sort()
# the last pipeline pass: from the last run of LM launches
lm = [x for x in k if "lm_kernel" in x[2]]
print("LM launches", len(lm))
# last 4 LM launches = last pass of the pipeline (4 batches)
t_end = lm[-1][1]
t0 = lm[-4][0]
# include the preparation of the first batch of that pass: kernels of fmpnp between previous LM end and t0
prev_end = lm[-5][1] if len(lm) > 4 else k[0][0]
win = [x for x in k if x[0] >= prev_end and x[1] <= t_end]
span = t_end - min(x[0] for x in win)
def busy(sel):
    iv = sorted((a, b) for a, b, n in win if sel(n))
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur: tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur: tot += cur[1] - cur[0]
    return tot, iv
lmb, lmiv = busy(lambda n: "lm_kernel" in n)
pkb, pkiv = busy(lambda n: "hwc" in n or "pack" in n)
gab, _ = busy(lambda n: "gather_ref" in n)
allb, _ = busy(lambda n: True)
ov = 0
for a, b in lmiv:
    for c, d in pkiv:
        ov += max(0, min(b, d) - max(a, c))
print(f"span {span/1e6:.2f} ms, busy(any) {allb/1e6:.2f}, LM {lmb/1e6:.2f}, pack {pkb/1e6:.2f}, gather {gab/1e6:.2f}, LM&pack overlap {ov/1e6:.2f} ms")
names = {}
for a, b, n in win:
    key = n.split("(")[0][:70]
    names.setdefault(key, [0, 0]); names[key][0] += 1; names[key][1] += b - a
for n, (c, t) in sorted(names.items(), key=lambda x: -x[1][1])[:12]:
    print(f"  {n:70s} {c:5d} {t/1e6:8.3f} ms")
PY
timeout -k 10 200 python3 "$REPO/tools/profile_pipeline_host.py" 4 128 2>&1 | grep -v amdgpu.ids | head -45
