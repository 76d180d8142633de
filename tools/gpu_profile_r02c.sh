#!/bin/bash
# Round-2 (third session) profiles after enabling the speculative gathers on the later wave of
# each SIMD: the workloads whose LM variant speculates, plus the no-spec leg and SQ counters.
export WORKLOADS="b128_easy|
b128_easy_nospec|--no-spec
b128_hard|--init hard
b128_hard_ratio0.8|--init hard --ratio 0.8
b128_easy_ratio0.8|--ratio 0.8"
export TRACE_BASE="--legs none --steps 100 --warmup 3 --event-every 1"
exec "$(dirname "$0")/gpu_profile_r02.sh"
