#!/bin/bash
# One GPU-box session: the driver's short bench line, the default bench line, then the
# -m gpu parity suite (TESTS selects files; default all).  Stops at the first GPU fault /
# abort / timeout (an ordinary test failure, rc 1, still reports).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r2}
mkdir -p $OUT
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $OUT/bench_short.log 2>&1
  rc=$?; echo "bench short rc=$rc"; tail -c 600 $OUT/bench_short.log; echo
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench_long.log 2>&1
  rc=$?; echo "bench long rc=$rc"; tail -c 600 $OUT/bench_long.log; echo
  [ $rc -eq 0 ] || exit $rc
fi
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 240 \
      --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_gpu.log | grep -v PASSED | head -30
  tail -3 $OUT/pytest_gpu.log
  exit $rc
fi
