#!/bin/bash
# Round-end profiles (part of tools/gpu_profile_all.sh), split for the gpurun time limit:
#   PART=lm    the LM workloads of the bench legs + SQ counters of the headline
#   PART=rest  the end-to-end pipelines, the RobotCar pyramids, the façade calls, TA/TD of the headline
# then tools/collect_profiles.sh TAG on the box, and a copy of profiles/TAG_* under gpurun_out/profiles_TAG/
# (gpurun returns gpurun_out/ only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export PYTHONUNBUFFERED=1
TAG=${TAG:-r05}
if [ "${PART:-lm}" = lm ]; then
WORKLOADS="b128_easy|
b128_hard|--init hard
b128_easy_ratio0.8|--ratio 0.8
b128_hard_ratio0.8|--init hard --ratio 0.8
b128_easy_nospec|--no-spec
b128_easy_bilinear|--sampling bilinear
b128_easy_layoutf|--layout f
b1024_easy|
b1024_easy_nomemo|--no-memo
b1024_easy_nomemo_bilinear|--no-memo --sampling bilinear" SQ=1 timeout -k 10 1000 bash tools/gpu_profile.sh \
    > gpurun_out/prof_lm.log 2>&1 || { tail -20 gpurun_out/prof_lm.log; exit 1; }
else
WINDOW=5 timeout -k 10 300 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe_w5.log 2>&1 || exit 1
timeout -k 10 300 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe.log 2>&1 || exit 1
ROBOTCAR=1 timeout -k 10 300 bash tools/gpu_profile_pipeline.sh > gpurun_out/prof_pipe_robotcar.log 2>&1 || exit 1
timeout -k 10 300 bash tools/gpu_profile_pyramid.sh 866 > gpurun_out/prof_pyr866.log 2>&1 || exit 1
timeout -k 10 300 bash tools/gpu_profile_pyramid.sh 295 > gpurun_out/prof_pyr295.log 2>&1 || exit 1
timeout -k 10 400 bash tools/gpu_profile_facade.sh > gpurun_out/prof_facade.log 2>&1 || exit 1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
    --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof/tatd" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --legs none \
    --steps 5 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/prof_tatd.log" 2>&1 ) || exit 1
fi
bash tools/collect_profiles.sh "$TAG" > /dev/null || exit 1
mkdir -p gpurun_out/profiles_$TAG && cp profiles/${TAG}_* gpurun_out/profiles_$TAG/ && ls gpurun_out/profiles_$TAG | wc -l
