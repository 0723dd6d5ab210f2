#!/bin/bash
# bf16 32x32 forward / dX tiles at 3 / 4 / 5 workgroups per CU (SACX_T32_BF_WGS, library variants)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abbfwgs
mkdir -p $OUT
for r in 1 2; do
  for v in bf3 bf4 bf5; do
    export SACX_LIBPATH=$PWD/tools/libvar/libsacx_$v.so
    timeout -k 10 240 python bench.py --config humanoid_bf16 --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 > $OUT/h_$v$r.log 2>&1 || exit $?
    timeout -k 10 240 python bench.py --config humanoid_bf16 --seeds-per-gpu 4 --steps 400 --warmup 50 --no-cpu-baseline --no-roofline > $OUT/h4_$v$r.log 2>&1 || exit $?
    echo "$v$r humanoid_bf16 $(grep -o '"value": [0-9.]*' $OUT/h_$v$r.log | head -1) x4 $(grep -o '"value": [0-9.]*' $OUT/h4_$v$r.log | head -1)"
  done
done
