#!/bin/bash
# Profiling set for one config (one GPU call): rocprofv3 kernel-trace stats of the one-seed
# bench, the PMC passes (tools/gpu_pmc.sh) and the per-launch workgroup timing of one update
# (tools/ktime_dump.py).  Outputs under gpurun_out/ (copy the ones to keep to profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=${CONFIG:-hc}
OUT=gpurun_out/prof_$CONFIG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/stats" -o s \
    -- python bench.py --config $CONFIG --steps 2000 --warmup 200 --no-cpu-baseline --packed-leg 0 > $OUT/bench_traced.log 2>&1
rc=$?; echo "rocprof stats rc=$rc"; tail -c 300 $OUT/bench_traced.log; echo; [ $rc -eq 0 ] || exit $rc
CONFIG=$CONFIG bash tools/gpu_pmc.sh || exit $?
timeout -k 10 200 python tools/ktime_dump.py $CONFIG > $OUT/ktime.txt 2>&1
rc=$?; echo "ktime rc=$rc"; tail -25 $OUT/ktime.txt; exit $rc
