#!/bin/bash
# rocprofv3 kernel-trace statistics of the single query (configs[1]) with the first-evaluation
# helpers (the default) and without them.
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
OUT="$REPO/gpurun_out/prof_b1"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for hv in 1 0; do
  FMPNP_HELPERS=$hv timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/h$hv" -o run -- python3 "$REPO/bench.py" --legs none --batch 1 --steps 200 --warmup 5 --event-every 1 > "$OUT/h$hv.json" 2> "$OUT/h$hv.err" || { tail -20 "$OUT/h$hv.err"; exit 1; }
  find "$OUT/h$hv" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats_h$hv.csv" \;
  rm -rf "$OUT/h$hv"
done
grep -h lm_kernel "$OUT"/kernel_stats_h*.csv | cut -c1-200
