#!/bin/bash
# Bench lines for the driver's own command and the other configs (SAC-EO at HC shapes, the
# C4 data-parallel mode at one rank, 8 packed seeds as the metric) -> gpurun_out/fin/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/fin
mkdir -p $OUT
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(grep -o '"value": [0-9.]*' $OUT/$tag.log | head -1)"
  return $rc
}
run driver_cmd --gpus 1 --steps 20 --warmup 5 &&
run hc_eo --config hc_eo --steps 1000 --warmup 100 &&
run dp1 --mode dp --steps 1000 --warmup 100 --no-cpu-baseline &&
run packed8 --seeds-per-gpu 8 --steps 1024 --warmup 128 --no-cpu-baseline
