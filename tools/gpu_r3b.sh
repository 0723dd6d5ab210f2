#!/bin/bash
# Round 3: drop-in tests + the GPU suite + drop-in A/B (SACX_SPEC 1/0) + smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dropin.py \
    > gpurun_out/dropin_test.log 2>&1; rc=$?; tail -6 gpurun_out/dropin_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 1 0 1 0; do
  SACX_SPEC=$s timeout -k 10 200 python tools/dropin_parts.py > gpurun_out/dropin_spec$s.log 2>&1 || exit $?
  echo "SPEC=$s"; tail -1 gpurun_out/dropin_spec$s.log
done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
