#!/bin/bash
# GPU test run for one gpurun call: tools/gpu_tests.sh <log-name> [pytest selectors...]
# (no selectors: the whole -m gpu suite).  Log under gpurun_out/<log-name>.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=$1; shift
sel=("$@"); [ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread -s "${sel[@]}" \
    > gpurun_out/$name.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 gpurun_out/$name.log; exit $rc
