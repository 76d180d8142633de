#!/bin/bash
# Interleaved A/B of library builds on the GPU box (bench.py legs, ms per launch):
#   tools/ab.sh NAME=LIB[@VAR=VAL...] ...     LIB: path of a libfmpnp.so, or "tree" (in-tree build);
#                                            @VAR=VAL: environment of that arm (e.g. @FMPNP_SPEC_CAP=2)
# env: REPS (3), STEPS (4000), LEGS (single,hard), EXTRA (more bench.py args).
# Per run one line: name, ms_per_step, kernel ms (HIP events), and each leg's ms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-3}); do
  for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}
    lib=${rest%%@*}; envs=""
    [ "$rest" != "$lib" ] && envs=$(echo "${rest#*@}" | tr '@' ' ')
    [ "$lib" = tree ] && lib=$PWD/featuremetric-pnp_amd/fmpnp/lib/libfmpnp.so
    env $envs FMPNP_LIB_PATH=$lib timeout -k 10 240 python3 bench.py --legs ${LEGS:-single,hard} --steps ${STEPS:-4000} \
        --warmup 20 ${EXTRA} > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err \
        || { echo "$name failed"; tail -5 gpurun_out/ab_$name.err; exit 1; }
    python3 - "$name" "gpurun_out/ab_$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
legs = [f"{k} {v['ms']}" for k, v in d.get("legs", {}).items() if "ms" in v]  # (the compact line)
print(f"{sys.argv[1]:>10s}  step {d['ms_per_step']:.4f}  kernel {d['roofline']['avg_kernel_ms']:.4f}  " + "  ".join(legs),
      flush=True)
PY
  done
done
