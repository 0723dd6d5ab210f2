#!/bin/bash
# Round 3: speculative drop-in for packed seeds: its tests, the GPU suite, --runs 8 timing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dropin.py tests/test_gpu_train.py \
    > gpurun_out/dropin_test.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/dropin_test.log | tail -14; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for alg in sac sac_imit; do
  SACX_LOCKSTEP_PROFILE=1 timeout -k 10 600 python -u tools/packed_runs_time.py 8 $alg 11000 > gpurun_out/packed_runs_$alg.log 2>&1 || exit $?
  grep -E "lockstep|speed-up|packed:|serial:" gpurun_out/packed_runs_$alg.log
done
