#!/bin/bash
# Sampler changes: rng_bench (split == one-kernel, per-phase ticks), the bit-exact sampler tests,
# then the whole GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/rng_bench > gpurun_out/rng_bench.log 2>&1; rc=$?; cat gpurun_out/rng_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "sampler or rng or golden or noise" > gpurun_out/pytest_rng.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_rng.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config humanoid_sac --no-cpu-baseline --packed-leg 0 > gpurun_out/bench_humanoid_sac.log 2>&1 || exit $?
python -c "import json; d=json.loads([l for l in open('gpurun_out/bench_humanoid_sac.log') if l.startswith('{')][-1]); print('humanoid_sac', d['value'], d['ms_per_step'])"
