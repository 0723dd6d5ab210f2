#!/bin/bash
# A/B of the bf16 32x32-tile occupancy: old = 6 workgroups per CU (spilling), new = 4 (default)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abbf
mkdir -p $OUT
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export SACX_LIBPATH=$PWD/tools/libvar/libsacx_old.so; else unset SACX_LIBPATH; fi
    timeout -k 10 240 python bench.py --config humanoid_bf16 --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 \
        > $OUT/hbf_$v$r.log 2>&1
    rc=$?; echo "humanoid_bf16 $v$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/hbf_$v$r.log | head -1)"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 240 python bench.py --config humanoid_bf16 --seeds-per-gpu 4 --steps 400 --warmup 50 --no-cpu-baseline --no-roofline \
        > $OUT/hbf4_$v$r.log 2>&1
    rc=$?; echo "humanoid_bf16 x4 $v$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/hbf4_$v$r.log | head -1)"; [ $rc -eq 0 ] || exit $rc
  done
done
