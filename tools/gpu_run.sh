#!/bin/bash
# One GPU session on the gpurun box: GPU tests (optionally a subset), then a headline bench.
#   tools/gpu_run.sh TAG [PYTEST_ARGS...]
# Logs: gpurun_out/<TAG>_pytest.log, gpurun_out/<TAG>_bench.json / .err.
# A test run that crashed (exit status other than 0/1: fault, abort, timeout) ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${1:-run}; shift
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -v --maxfail=${MAXFAIL:-20} \
      --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?
  tail -n 40 gpurun_out/${TAG}_pytest.log
  if [ $rc -gt 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-300} python -u bench.py --steps ${STEPS:-2000} --legs ${LEGS:-none} \
      > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  rc=$?
  tail -c 3000 gpurun_out/${TAG}_bench.json; tail -n 5 gpurun_out/${TAG}_bench.err
  exit $rc
fi
