#!/bin/bash
# Packed-seed (K = 8) variants of the update plan: tile shape, fused actor head, XCD map.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/multi_seed.py ${KS:-8} 2>&1 | grep config || exit 1; }
run SACX_T32=2
run SACX_T32=0
run SACX_T32=1
run SACX_T32=2 SACX_FUSE_HEAD=0
run SACX_T32=0 SACX_FUSE_HEAD=0
