#!/bin/bash
# Round-end measurement set (one GPU call): the default bench line (roofline + CPU
# baseline), the rocprofv3 kernel-trace stats of the same command, and the PMC passes
# that feed roofline.traffic.  Outputs under gpurun_out/refresh/ (copy to profiles/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/refresh
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_hc.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench_hc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o hc \
    -- python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --packed-leg 0 > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/prof -name "*kernel_stats*" | head -3
bash tools/gpu_pmc.sh
