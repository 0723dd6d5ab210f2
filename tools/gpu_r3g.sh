#!/bin/bash
# Round-3 late check: the GPU suite, smoke, the default bench line, --runs 8 packed vs serial.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r3g
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3g/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r3g/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3g/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/r3g/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r3g/bench_hc.log 2>&1
rc=$?; echo "bench rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r3g/bench_hc.log | head -1) $(grep -o '"drop_in_loop": {"updates_per_s": [0-9.]*' gpurun_out/r3g/bench_hc.log)"; [ $rc -eq 0 ] || exit $rc
for alg in sac sac_imit; do
  SACX_LOCKSTEP_PROFILE=1 timeout -k 10 600 python -u tools/packed_runs_time.py 8 $alg 11000 > gpurun_out/r3g/packed_runs_$alg.log 2>&1 || exit $?
  grep -E "lockstep|speed-up" gpurun_out/r3g/packed_runs_$alg.log
done
