#!/bin/bash
# The one-call façade's packed window (fmpnp_feature_pnp window_radius; FMPNP_FACADE_WINDOW) against
# the full pack: ms per call and the calls re-run fully packed, cfg2 and the RobotCar shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
for rep in 1 2; do
  for w in 0 3 4 5 6 8; do
    FMPNP_FACADE_WINDOW=$w timeout -k 10 200 python3 tools/facade_call.py cfg2 robotcar_n295 robotcar_n866 --calls 24 2>/dev/null \
      | python3 -c "import json,sys; print('window $w', ' '.join(f\"{d['shape_name']} {d['ms_per_call']} (reruns {d['window_reruns']})\" for d in map(json.loads, sys.stdin)))" || exit 1
  done
done
