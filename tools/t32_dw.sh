#!/bin/bash
# 32x32 tiles for every launch (SACX_T32=1, dW + Adam included) vs forward / dX only (2)
# on the packed / wide configs: t32_dw.sh "<config> <seeds>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfgk in "$@"; do
  set -- $cfgk
  for t in 2 1; do
    echo "T32=$t $(SACX_T32=$t MS_CONFIG=$1 timeout -k 10 150 python tools/multi_seed.py $2 2>&1 | grep config)" || exit 1
  done
done
