#!/bin/bash
# HBM bytes per query of the end-to-end pipeline (bench.py end_to_end): separate FETCH_SIZE and
# WRITE_SIZE passes of tools/pipeline_run.py (kernel trace only, MI355X_MICROARCH.md), summed over
# the fmpnp kernels (the f-only pack, the reference gather, the LM launches) per query processed.
# Output: gpurun_out/prof/pipeline/summary.json (copy to profiles/rNN_pmc_pipeline.json);
# WINDOW=r: the windowed packs of radius r (gpurun_out/prof/pipeline_w<r>/).
set -o pipefail
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
D="$REPO/gpurun_out/prof/pipeline${WINDOW:+_w$WINDOW}${ROBOTCAR:+_robotcar}"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/trace" -o run -- python3 "$REPO/tools/pipeline_run.py" 2 > "$D/run.log" 2>&1 || { tail -20 "$D/run.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 "$REPO/tools/pipeline_run.py" 2 > /dev/null 2> "$D/fetch.err" || { tail -20 "$D/fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 "$REPO/tools/pipeline_run.py" 2 > /dev/null 2> "$D/write.err" || { tail -20 "$D/write.err"; exit 1; }
python3 "$REPO/tools/pmc_pipeline_summary.py" "$D" "$(grep -o 'queries [0-9]*' "$D/run.log" | cut -d' ' -f2)" || exit 1
rm -rf "$D/pmc_fetch" "$D/pmc_write"
