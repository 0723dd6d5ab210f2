#!/bin/bash
# Sampler batch (updates per k_rng launch, SACX_NBATCH) vs the one-seed update rate.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in hc humanoid_sac; do
  for nb in 2 4 8; do
    echo "NBATCH=$nb $(SACX_NBATCH=$nb MS_CONFIG=$cfg timeout -k 10 150 python tools/multi_seed.py 1 2>&1 | grep config)" || exit 1
  done
done
