#!/bin/bash
# A/B of two builds of libsacx, alternating runs:
#   ab_lib.sh <B library path> <config> <rounds> <packed seeds K...>
# A = the in-tree sac-expert_amd/lib/libsacx.so, B = SACX_LIBPATH=<B library path>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
lib=$1; cfg=$2; rounds=$3; shift 3
for r in $(seq "$rounds"); do
  for k in "$@"; do
    echo "A: $(MS_CONFIG=$cfg timeout -k 10 150 python tools/multi_seed.py "$k" 2>&1 | grep config)" || exit 1
    echo "B: $(SACX_LIBPATH=$lib MS_CONFIG=$cfg timeout -k 10 150 python tools/multi_seed.py "$k" 2>&1 | grep config)" || exit 1
  done
done
