#!/bin/bash
# A/B of the drop-in loop's speculative sampler (SACX_SPEC=1 vs 0, alternating), after its
# bit-identity test; then smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dropin.py \
    > gpurun_out/dropin_test.log 2>&1; rc=$?; tail -3 gpurun_out/dropin_test.log; [ $rc -eq 0 ] || exit $rc
for s in 1 0 1 0; do
  SACX_SPEC=$s timeout -k 10 200 python tools/dropin_parts.py > gpurun_out/dropin_spec$s.log 2>&1 || exit $?
  echo "SPEC=$s"; tail -3 gpurun_out/dropin_spec$s.log
done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
