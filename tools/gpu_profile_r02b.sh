#!/bin/bash
# Round-2 (second session) profiles at the current build: speculation compiled out, the
# bilinear cell memo.  Same passes as tools/gpu_profile_r02.sh.
export WORKLOADS="b128_easy|
b128_hard|--init hard
b128_hard_ratio0.8|--init hard --ratio 0.8
b128_easy_ratio0.8|--ratio 0.8
b128_easy_nomemo|--no-memo
b128_easy_bilinear|--sampling bilinear
b128_easy_nomemo_bilinear|--sampling bilinear --no-memo
b128_easy_layoutf|--layout f
b1024_easy|"
export TRACE_BASE="--legs none --steps 100 --warmup 3 --event-every 1"
exec "$(dirname "$0")/gpu_profile_r02.sh"
