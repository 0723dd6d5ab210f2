#!/bin/bash
# Humanoid-shaped configs with 16x16 vs 32x32 forward / dX tiles (one seed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in humanoid_sac humanoid_eo humanoid_bf16; do
  for t in 0 2; do
    SACX_T32=$t timeout -k 10 200 python bench.py --config $cfg --steps 1000 --warmup 100 --no-cpu-baseline \
      --no-roofline --packed-leg 0 > gpurun_out/t32_${cfg}_$t.log 2>&1 || exit 1
    echo "$cfg T32=$t $(tail -1 gpurun_out/t32_${cfg}_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("model_fit",{}).get("steps_per_s"))')"
  done
done
