#!/bin/bash
# A/B: the default dW tile rule (B) against 32x32 dW tiles for every dW launch (C: SACX_DW_ROUND=1)
# -> gpurun_out/abdw2/<config>_<arm><round>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abdw2
mkdir -p $OUT
for r in 1 2; do
  for c in ${CONFIGS:-humanoid_bf16 hc}; do
    for arm in B C; do
      if [ $arm = C ]; then export SACX_DW_ROUND=1; else unset SACX_DW_ROUND; fi
      timeout -k 10 240 python bench.py --config $c --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline --no-roofline --packed-leg 0 \
          > $OUT/${c}_$arm$r.log 2>&1
      rc=$?; echo "$c $arm$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/${c}_$arm$r.log | head -1)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
