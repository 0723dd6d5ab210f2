#!/bin/bash
# A/B of the dW tile rule on the Humanoid configs: A = 16x16 dW tiles everywhere on one-seed
# plans (SACX_DW_ROUND huge), B = the default (32x32 for launches past one round of residency).
# Alternating, two rounds -> gpurun_out/abdw/<config>_<arm><round>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/abdw
mkdir -p $OUT
for r in 1 2; do
  for c in ${CONFIGS:-humanoid_sac humanoid_bf16 humanoid_eo}; do
    for arm in A B; do
      if [ $arm = A ]; then export SACX_DW_ROUND=100000000; else unset SACX_DW_ROUND; fi
      timeout -k 10 240 python bench.py --config $c --steps ${STEPS:-1000} --warmup 100 --no-cpu-baseline --packed-leg 0 \
          > $OUT/${c}_$arm$r.log 2>&1
      rc=$?; echo "$c $arm$r rc=$rc $(grep -o '"value": [0-9.]*' $OUT/${c}_$arm$r.log | head -1)"
      [ $rc -eq 0 ] || exit $rc
    done
  done
done
