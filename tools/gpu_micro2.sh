#!/bin/bash
# Isolated kernel timings (graph replay) for the GEMM and row kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/gemm_bench > gpurun_out/micro_gemm.log 2>&1; rc=$?; cat gpurun_out/micro_gemm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/rows_bench > gpurun_out/micro_rows.log 2>&1; rc=$?; cat gpurun_out/micro_rows.log
exit $rc
