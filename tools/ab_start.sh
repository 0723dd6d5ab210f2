#!/bin/bash
# The driver's command (--steps 20 --warmup 5) on the session-start library vs the current one,
# alternating, three rounds; then one 2,000-step line each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abstart
mkdir -p $OUT
for r in 1 2 3; do
  for v in start now; do
    if [ $v = start ]; then export SACX_LIBPATH=$PWD/tools/libvar/libsacx_start.so; else unset SACX_LIBPATH; fi
    timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --packed-leg 0 > $OUT/d_$v$r.log 2>&1 || exit $?
    echo "driver cmd $v$r $(grep -o '"value": [0-9.]*' $OUT/d_$v$r.log | head -1) $(grep -o '"ms_per_step": [0-9.]*' $OUT/d_$v$r.log | head -1)"
  done
done
for v in start now; do
  if [ $v = start ]; then export SACX_LIBPATH=$PWD/tools/libvar/libsacx_start.so; else unset SACX_LIBPATH; fi
  timeout -k 10 240 python bench.py --no-cpu-baseline --packed-leg 0 > $OUT/l_$v.log 2>&1 || exit $?
  echo "2000 steps $v $(grep -o '"value": [0-9.]*' $OUT/l_$v.log | head -1)"
done
