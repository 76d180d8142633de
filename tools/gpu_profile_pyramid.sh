#!/bin/bash
# Per-level HBM bytes of the RobotCar channel pyramid (bench.py pyramid_robotcar_1664) at N points:
# kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of tools/pyramid_run.py, summarised per level
# (the LM launches in dispatch order: REPS per level) by tools/pmc_pyramid_summary.py.
#   usage: tools/gpu_profile_pyramid.sh N   -> gpurun_out/prof/pyramid_n<N>/summary.json
set -o pipefail
N=${1:-866}
REPO="${GRAFT_REPO_ROOT:-$(pwd)}"
D="$REPO/gpurun_out/prof/pyramid_n$N"
mkdir -p "$D"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$D/trace" -o run -- python3 "$REPO/tools/pyramid_run.py" "$N" 4 > "$D/run.log" 2>&1 || { tail -20 "$D/run.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$D/pmc_fetch" -o run -- python3 "$REPO/tools/pyramid_run.py" "$N" 4 > /dev/null 2> "$D/fetch.err" || { tail -20 "$D/fetch.err"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$D/pmc_write" -o run -- python3 "$REPO/tools/pyramid_run.py" "$N" 4 > /dev/null 2> "$D/write.err" || { tail -20 "$D/write.err"; exit 1; }
python3 "$REPO/tools/pmc_pyramid_summary.py" "$D" "$N" 4 || exit 1
rm -rf "$D/pmc_fetch" "$D/pmc_write"
