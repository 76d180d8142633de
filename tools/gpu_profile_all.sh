#!/bin/bash
# Every PMC-backed roofline bench.py reports, for the current sources (one GPU call): the LM
# workloads of the bench legs (tools/gpu_profile.sh, SQ counters of the headline included), the
# end-to-end pipeline with windowed and full packs, and the RobotCar pyramid at N = 866 and 295.
# Summaries land under gpurun_out/prof/; tools/collect_profiles.sh RNN copies them to profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export PYTHONUNBUFFERED=1
WORKLOADS="b128_easy|
b128_hard|--init hard
b128_easy_ratio0.8|--ratio 0.8
b128_hard_ratio0.8|--init hard --ratio 0.8
b128_easy_nospec|--no-spec
b128_easy_bilinear|--sampling bilinear
b128_easy_layoutf|--layout f
b1024_easy|
b1024_easy_nomemo|--no-memo
b1024_easy_nomemo_bilinear|--no-memo --sampling bilinear" SQ=1 timeout -k 10 1500 bash tools/gpu_profile.sh \
    > gpurun_out/prof_lm.log 2>&1 || { tail -20 gpurun_out/prof_lm.log; exit 1; }
WINDOW=5 timeout -k 10 400 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe_w5.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe.log 2>&1 || exit 1
ROBOTCAR=1 timeout -k 10 400 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe_robotcar.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_profile_pyramid.sh 866 > gpurun_out/prof_pyr866.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_profile_pyramid.sh 295 > gpurun_out/prof_pyr295.log 2>&1 || exit 1
timeout -k 10 500 bash tools/gpu_profile_facade.sh > gpurun_out/prof_facade.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv \
    -d "$GRAFT_REPO_ROOT/gpurun_out/prof/tatd" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --legs none --steps 5 \
    --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_tatd.log" 2>&1
echo "profiles done"
