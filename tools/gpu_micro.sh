#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/microbench > gpurun_out/micro.log 2>&1; rc=$?; cat gpurun_out/micro.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -k "model_fit" > gpurun_out/pytest_mfit.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_mfit.log; exit $rc
