#!/bin/bash
# A/B of the f-only pack kernels: multi-row LDS tiles (FMPNP_PACK_F_ROWS=1) vs LDS tiles (=0)
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_window_pack.py tests/test_layout_f.py tests/test_batch_prep.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/packreg_tests.log 2>&1 || { tail -30 gpurun_out/packreg_tests.log; exit 1; }
tail -2 gpurun_out/packreg_tests.log
for rep in 1 2; do
  for reg in 0 1; do
    FMPNP_PACK_F_ROWS=$reg timeout -k 10 200 python bench.py --legs pack,pipeline --steps 200 --warmup 5 --detail gpurun_out/packab_${reg}_${rep}.json > gpurun_out/packab_${reg}_${rep}.line 2> gpurun_out/packab_${reg}_${rep}.err || { tail gpurun_out/packab_${reg}_${rep}.err; exit 1; }
    python - "$reg" "$rep" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/packab_{sys.argv[1]}_{sys.argv[2]}.json"))
e = d["end_to_end"]
print(f"rows={sys.argv[1]} rep={sys.argv[2]} pack_f {d['pack_f']['ms']} ms {d['pack_f']['frac_of_peak']}  e2e {e['queries_per_s']} q/s steady {e['steady_state_queries_per_s']} hard {e['hard_init']['queries_per_s']} full {e['full_pack']['queries_per_s']} same {e['identical_to_full_pack']} robotcar {e['robotcar_1664'].get('queries_per_s')}")
PY
  done
done
