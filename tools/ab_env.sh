#!/bin/bash
# A/B of one env setting on the one-seed HC rate, alternating runs: ab_env.sh "VAR=val" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${2:-2}); do
  echo "A: $(timeout -k 10 120 python tools/multi_seed.py 1 2>&1 | grep config)" || exit 1
  echo "B $1: $(env $1 timeout -k 10 120 python tools/multi_seed.py 1 2>&1 | grep config)" || exit 1
done
