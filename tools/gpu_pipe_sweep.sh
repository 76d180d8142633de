#!/bin/bash
# End-to-end pipeline throughput for several batch shapes (tools/bench_pipeline.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "4 64" "4 128" "2 256" "8 128"; do
  timeout -k 10 300 python3 tools/bench_pipeline.py $cfg > gpurun_out/pipe_$(echo $cfg | tr ' ' x).json 2> gpurun_out/pipe.err || { tail gpurun_out/pipe.err; exit 1; }
  echo "$cfg: $(tail -c 400 gpurun_out/pipe_$(echo $cfg | tr ' ' x).json)"
done
