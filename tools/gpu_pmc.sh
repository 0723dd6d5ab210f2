#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) over a short bench of
# config ${CONFIG:-hc}; summary -> profiles/pmc_<config>.json (+ copy in gpurun_out/).
# Pass 4 is the MFMA pipe: SQ_VALU_MFMA_BUSY_CYCLES (cycles the matrix pipe is busy, summed
# over SIMDs) with GRBM_GUI_ACTIVE (GPU-busy cycles) for the utilisation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=${CONFIG:-hc}
OUT=gpurun_out/pmc_$CONFIG
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$PWD/$OUT" -o "p$i" \
      -- python bench.py --config $CONFIG --steps 200 --warmup 20 --no-cpu-baseline --no-roofline --packed-leg 0 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"; tail -1 $OUT/p$i.log
  [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py $OUT $CONFIG "${PMC_TAG:-$CONFIG}" gpurun_out/pmc_$CONFIG.json
