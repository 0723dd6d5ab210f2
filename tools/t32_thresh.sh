#!/bin/bash
# 16x16 vs 32x32 forward / dX tiles at small seeds x batch (HC shapes, B = 256): where the
# tile32 threshold (seeds x B >= 1024) should sit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in 1 2 4; do
  for t in 0 2; do
    echo "K=$k T32=$t $(SACX_T32=$t MS_CONFIG=hc timeout -k 10 150 python tools/multi_seed.py $k 2>&1 | grep config)" || exit 1
  done
done
