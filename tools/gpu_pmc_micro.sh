#!/bin/bash
# PMC passes over the isolated GEMM microbenchmark (one counter group per run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcm
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
           "SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmcm" -o "m$i" \
      -- ./tools/gemm_bench > gpurun_out/pmcm/m$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; tail -2 gpurun_out/pmcm/m$i.log
  [ $rc -eq 0 ] || exit $rc
done
ls gpurun_out/pmcm
