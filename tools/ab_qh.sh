#!/bin/bash
# A/B of the fp32 32x32 dX + Q-head-row tiles' occupancy: old = 6 workgroups per CU (17-18 VGPRs
# spilled), new = 5 (default); Humanoid one seed and 4 seeds, HC 8 packed seeds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abqh
mkdir -p $OUT
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export SACX_LIBPATH=$PWD/tools/libvar/libsacx_bf4.so; else unset SACX_LIBPATH; fi
    timeout -k 10 240 python bench.py --config humanoid_sac --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 > $OUT/hs_$v$r.log 2>&1 || exit $?
    timeout -k 10 240 python bench.py --config humanoid_sac --seeds-per-gpu 4 --steps 400 --warmup 50 --no-cpu-baseline --no-roofline > $OUT/hs4_$v$r.log 2>&1 || exit $?
    timeout -k 10 240 python bench.py --seeds-per-gpu 8 --steps 1024 --warmup 100 --no-cpu-baseline --no-roofline > $OUT/hc8_$v$r.log 2>&1 || exit $?
    echo "$v$r humanoid $(grep -o '"value": [0-9.]*' $OUT/hs_$v$r.log | head -1) humanoid x4 $(grep -o '"value": [0-9.]*' $OUT/hs4_$v$r.log | head -1) hc x8 $(grep -o '"value": [0-9.]*' $OUT/hc8_$v$r.log | head -1)"
  done
done
