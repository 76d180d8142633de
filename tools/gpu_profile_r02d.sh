#!/bin/bash
# Round-2 (third session) profiles of the workloads whose kernel variant changed when the
# speculation moved into its own variants: the no-speculation leg and layout F.
export WORKLOADS="b128_easy_nospec|--no-spec
b128_easy_layoutf|--layout f"
export TRACE_BASE="--legs none --steps 100 --warmup 3 --event-every 1"
exec "$(dirname "$0")/gpu_profile_r02.sh"
