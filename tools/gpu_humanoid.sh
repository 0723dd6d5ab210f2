#!/bin/bash
# Humanoid bench lines (SAC fp32, SAC bf16 operands, SAC-EO) -> gpurun_out/hum/<config>.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/hum
mkdir -p $OUT
for c in humanoid_sac humanoid_bf16 humanoid_eo; do
  timeout -k 10 300 python bench.py --config $c --steps 1000 --warmup 100 > $OUT/$c.log 2>&1
  rc=$?; echo "$c rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$c.log | head -1)"
  [ $rc -eq 0 ] || exit $rc
done
