#!/bin/bash
# Round-end evidence on the GPU box, in the driver's order: GPU tests, smoke(), the default bench
# line (every leg), then the headline's rocprofv3 kernel stats + FETCH/WRITE passes.
#   tools/gpu_final.sh TAG     -> gpurun_out/<TAG>_pytest.log, <TAG>_smoke.log, <TAG>_bench.json,
#                                 gpurun_out/prof/b128_easy/{summary.json,kernel_stats.csv}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${1:-final}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/${TAG}_pytest.log
[ $rc -le 1 ] || { echo "pytest exit $rc"; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { tail -n 5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { tail -n 5 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench.json
WORKLOADS="b128_easy|" timeout -k 10 400 bash tools/gpu_profile.sh
