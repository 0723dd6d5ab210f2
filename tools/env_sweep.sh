#!/bin/bash
# HIP runtime knobs vs the one-seed HC update rate (tools/multi_seed.py K=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { echo "== ${*:-baseline}"; env "$@" timeout -k 10 120 python tools/multi_seed.py 1 2>&1 | grep config || exit 1; }
run
run HIP_FORCE_DEV_KERNARG=1
run HIP_FORCE_DEV_KERNARG=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1
run HSA_ENABLE_SDMA=0
run
