#!/bin/bash
# Round-3 final set: the GPU suite, smoke, then the measurement refresh (bench line, rocprofv3
# stats of the same command, HC ktime, PMC passes) and the Humanoid lines + Humanoid ktime.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_refresh3.sh || exit $?
for c in humanoid_sac humanoid_bf16 humanoid_eo; do
  timeout -k 10 300 python bench.py --config $c --steps 1000 --warmup 100 --no-cpu-baseline > gpurun_out/refresh3/$c.log 2>&1
  rc=$?; echo "$c rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/refresh3/$c.log | head -1)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python tools/ktime_dump.py humanoid_sac > gpurun_out/refresh3/humanoid_sac_ktime.txt 2>&1 || exit $?
tail -1 gpurun_out/refresh3/humanoid_sac_ktime.txt
