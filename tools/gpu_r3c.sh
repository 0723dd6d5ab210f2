#!/bin/bash
# Round 3: split sampler check (rng_bench), GPU suite, drop-in A/B, Humanoid SAC / SAC-EO benches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/rng_bench > gpurun_out/rng_bench.log 2>&1; rc=$?; cat gpurun_out/rng_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for s in 1 0; do
  SACX_SPEC=$s timeout -k 10 200 python tools/dropin_parts.py > gpurun_out/dropin_spec$s.log 2>&1 || exit $?
  echo "SPEC=$s"; tail -1 gpurun_out/dropin_spec$s.log
done
for c in humanoid_sac humanoid_eo; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --packed-leg 0 > gpurun_out/bench_$c.log 2>&1 || exit $?
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_$c.log') if l.startswith('{')][-1]); print('$c', d['value'], d['ms_per_step'])"
done
