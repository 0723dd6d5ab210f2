#!/bin/bash
# A/B of the 32x32 tiles' k slabs per load group (SACX_T32_NS, SACX_T32_WGS workgroups per CU)
# through library variants (SACX_LIBPATH): base (1 / 6), ns2 (2 / 5), ns4 (4 / 4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abns
mkdir -p $OUT
for r in 1 2; do
  for c in humanoid_sac humanoid_bf16; do
    for v in base ns2 ns4; do
      if [ $v = base ]; then unset SACX_LIBPATH; else export SACX_LIBPATH=$PWD/tools/libvar/libsacx_$v.so; fi
      timeout -k 10 240 python bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 \
          > $OUT/${c}_$v$r.log 2>&1
      rc=$?; echo "$c $v$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/${c}_$v$r.log | head -1)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
for v in base ns2 ns4; do
  if [ $v = base ]; then unset SACX_LIBPATH; else export SACX_LIBPATH=$PWD/tools/libvar/libsacx_$v.so; fi
  timeout -k 10 240 python bench.py --config humanoid_sac --seeds-per-gpu 4 --steps 400 --warmup 50 --no-cpu-baseline --no-roofline \
      > $OUT/hum4_$v.log 2>&1
  rc=$?; echo "humanoid_sac x4 seeds $v rc=$rc $(grep -o '"value": [0-9.]*' $OUT/hum4_$v.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
