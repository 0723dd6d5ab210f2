#!/bin/bash
# Round-3 measurement set: default bench line, rocprofv3 kernel-trace stats of the same command,
# PMC passes (tools/gpu_pmc.sh), HC ktime.  -> gpurun_out/refresh3/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/refresh3
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench_hc.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/bench_hc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o hc \
    -- python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --packed-leg 0 > $OUT/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/ktime_dump.py hc > $OUT/hc_ktime.txt 2>&1 || exit $?
tail -1 $OUT/hc_ktime.txt
bash tools/gpu_pmc.sh
