#!/bin/bash
# A/B of the speculative gathers on wide channel slices (FMPNP_SPEC_MAXC: the widest slice that
# speculates; default 256 fp32 channels): the RobotCar façade call (B = 1, three levels of C = 1024 /
# 512 / 128) and the batched RobotCar pyramid (B = 32, bench.py pyramid1664 leg).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for i in 1 2; do
  for c in 256 1024; do
    FMPNP_SPEC_MAXC=$c timeout -k 10 200 python3 tools/facade_call.py robotcar_n295 robotcar_n866 --calls 24 2>/dev/null \
      | python3 -c "import json,sys; print('maxc $c facade', ' '.join(f\"{d['shape_name']} {d['ms_per_call']}\" for d in map(json.loads, sys.stdin)))" || exit 1
    FMPNP_SPEC_MAXC=$c timeout -k 10 300 python3 bench.py --legs pyramid1664 --steps 200 --warmup 5 --detail gpurun_out/pyr_$c.json 2>/dev/null \
      | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); L=d['legs']; print('maxc $c pyramid B=32', 'n866', L['pyramid_robotcar_1664']['ms'], 'n295', L['pyramid_robotcar_1664.median_query_n295']['ms'])" || exit 1
  done
done
