#!/bin/bash
# A/B of the sampler batch (updates per k_rng launch) on the current build, HC one seed
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/nbab
for r in 1 2; do
for nb in 4 8 2; do
  SACX_NBATCH=$nb timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --packed-leg 0 > gpurun_out/nbab/out.log 2>&1 || exit 1
  echo "$r nbatch=$nb $(python -c "import json,sys; [print(json.loads(l)['value']) for l in open(sys.argv[1]) if l.startswith('{')]" gpurun_out/nbab/out.log)"
done; done
