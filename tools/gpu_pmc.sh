#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc" -o "p$i" \
      -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-roofline > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; tail -2 gpurun_out/pmc/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
ls gpurun_out/pmc
