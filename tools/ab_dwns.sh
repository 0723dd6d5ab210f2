#!/bin/bash
# A/B of the 32x32 dW + Adam tiles' k slabs per load group (SACX_T32_DW_NS 1 / 2 / 4, library
# variants): Humanoid SAC one seed (critic.adam on 32x32) and 4 packed seeds, SAC-EO
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abdwns
mkdir -p $OUT
for r in 1 2; do
  for v in dw1 dw2 dw4; do
    export SACX_LIBPATH=$PWD/tools/libvar/libsacx_$v.so
    timeout -k 10 240 python bench.py --config humanoid_sac --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 > $OUT/hs_$v$r.log 2>&1 || exit $?
    timeout -k 10 240 python bench.py --config humanoid_sac --seeds-per-gpu 4 --steps 400 --warmup 50 --no-cpu-baseline --no-roofline > $OUT/hs4_$v$r.log 2>&1 || exit $?
    timeout -k 10 240 python bench.py --config humanoid_eo --steps 1000 --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 > $OUT/he_$v$r.log 2>&1 || exit $?
    echo "$v$r humanoid $(grep -o '"value": [0-9.]*' $OUT/hs_$v$r.log | head -1) x4 $(grep -o '"value": [0-9.]*' $OUT/hs4_$v$r.log | head -1) eo $(grep -o '"value": [0-9.]*' $OUT/he_$v$r.log | head -1)"
  done
done
