#!/bin/bash
# Model-fit (A16) timing at HC and Humanoid shapes + a kernel trace of the HC fit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mfit${TAG:-}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/model_fit_time.py hc_eo 512 > $OUT/hc.log 2>&1 || { cat $OUT/hc.log; exit 1; }
cat $OUT/hc.log
timeout -k 10 200 python tools/model_fit_time.py humanoid_eo 256 > $OUT/hum.log 2>&1 || { cat $OUT/hum.log; exit 1; }
cat $OUT/hum.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$OUT/trace" -o mfit \
    -- python tools/model_fit_time.py hc_eo 128 > $OUT/trace.log 2>&1 || { tail $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_view.py "$f" 24 k_mgather > $OUT/hc_trace_step.txt; cat $OUT/hc_trace_step.txt
