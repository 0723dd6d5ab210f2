#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench.  Stops at the first
# GPU fault / abort / timeout (only ordinary test failures, rc 1, continue).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HIP_LAUNCH_BLOCKING=${HIP_LAUNCH_BLOCKING:-0}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "${PROF:-}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o "$PROF" \
      -- python bench.py --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_bench.log; find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
