#!/bin/bash
# Round 3: --runs 8 packed vs serial wall time (sac and sac_imit), Humanoid ktime, HC bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for alg in sac sac_imit; do
  timeout -k 10 400 python -u tools/packed_runs_time.py 8 $alg > gpurun_out/packed_runs_$alg.log 2>&1; rc=$?
  tail -6 gpurun_out/packed_runs_$alg.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python tools/ktime_dump.py humanoid_sac > gpurun_out/hum_ktime.txt 2>&1 || exit $?
tail -3 gpurun_out/hum_ktime.txt
