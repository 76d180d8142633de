#!/bin/bash
# Batch scaling on one GPU (north_star: "near-linear batch scaling"): the headline workload (cfg2,
# memoised, easy start) at B queries per launch, one bench.py run per B (no legs).
#   tools/batch_sweep.sh [B ...]  -> gpurun_out/batch_sweep.jsonl (one summary line per B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
out=gpurun_out/batch_sweep.jsonl
: > "$out"
for B in ${@:-1 8 32 64 128 192 256 384 512 768 1024}; do
  steps=$(( 256000 / B )); [ $steps -lt 200 ] && steps=200; [ $steps -gt 20000 ] && steps=20000
  timeout -k 10 300 python3 bench.py --legs none --batch $B --steps $steps --warmup 5 \
      > gpurun_out/bs_$B.json 2> gpurun_out/bs_$B.err || { echo "B=$B failed"; tail -5 gpurun_out/bs_$B.err; exit 1; }
  python3 - "$B" "gpurun_out/bs_$B.json" >> "$out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(json.dumps({"batch": int(sys.argv[1]), "ms_per_launch": d["ms_per_step"], "pose_refinements_per_s": d["value"],
                  "kernel": r.get("kernel"), "kernel_ms": r.get("avg_kernel_ms"), "statuses": d.get("statuses")}))
PY
  tail -n 1 "$out"
done
