#!/bin/bash
# A/B of one environment switch on the same build: alternating bench runs with and without
# $AB_VAR=0 (the switch's "off" value), then (unless SKIP_TESTS) the -m gpu suite.
# usage: AB_VAR=SACX_FOLD_HBW [ROUNDS=2] [BENCH_ARGS=...] bash tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
BA="--no-cpu-baseline --packed-leg 0 ${BENCH_ARGS:-}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in on off; do
    if [ $v = off ]; then export $AB_VAR=0; else unset $AB_VAR; fi
    timeout -k 10 300 python bench.py $BA > $OUT/bench_${v}_$r.log 2>&1
    rc=$?
    python - $OUT/bench_${v}_$r.log $v $r <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); ro = d.get("roofline") or {}
        print(sys.argv[2], sys.argv[3], d["value"], ro.get("avg_launch_us"), ro.get("launches_per_update"))
PY
    [ $rc -eq 0 ] || exit $rc
  done
done
unset $AB_VAR
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 240 \
      --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.log | head -30
  tail -3 $OUT/pytest_gpu.log
  exit $rc
fi
