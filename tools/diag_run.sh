#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "relu 256 11 0.01" "tanh 128 21 0.0"; do
  for m in eager g1 g8; do
    timeout -k 10 120 python tools/diag_graph.py $m $cfg >> gpurun_out/diag.log 2>&1 || { echo "FAIL $m $cfg rc=$?"; exit 1; }
  done
  SACX_NO_FORK=1 timeout -k 10 120 python tools/diag_graph.py g8 $cfg >> gpurun_out/diag.log 2>&1 || { echo "FAIL nofork $cfg"; exit 1; }
done
grep '^{' gpurun_out/diag.log
