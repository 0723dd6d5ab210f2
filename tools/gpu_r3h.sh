#!/bin/bash
# Round-3 closing check: the GPU suite, smoke, the default bench line, the Humanoid lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r3h
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench_hc.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_hc.log | head -1) $(grep -o '"drop_in_loop": {"updates_per_s": [0-9.]*' $OUT/bench_hc.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.log 2>&1
rc=$?; echo "driver cmd rc=$rc $(grep -o '"value": [0-9.]*' $OUT/bench_driver_cmd.log | head -1)"; [ $rc -eq 0 ] || exit $rc
for c in humanoid_sac humanoid_bf16 humanoid_eo; do
  timeout -k 10 300 python bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline > $OUT/$c.log 2>&1
  rc=$?; echo "$c rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$c.log | head -1)"; [ $rc -eq 0 ] || exit $rc
done
