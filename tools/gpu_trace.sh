#!/bin/bash
# Kernel trace of a short bench (queue assignment / gaps of the captured graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/trace
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/trace" -o "${TAG:-t}" \
    -- python bench.py --steps 300 --warmup 50 --no-cpu-baseline --no-roofline > gpurun_out/trace/${TAG:-t}.log 2>&1
rc=$?; tail -2 gpurun_out/trace/${TAG:-t}.log; exit $rc
