#!/bin/bash
# Alternating A/B of environment settings on the current build (HC one seed, no CPU leg):
#   ENVS="X=1 SACX_FOO=1" ROUNDS=2 bash tools/env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/envab
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS:-X=1}; do
    env ${e//,/ } timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --packed-leg 0 ${BENCH_ARGS:-} \
        > gpurun_out/envab/out.log 2>&1 || exit 1
    echo "$r [$e] $(python -c "import json,sys; [print(json.loads(l)['value']) for l in open(sys.argv[1]) if l.startswith('{')]" gpurun_out/envab/out.log)"
  done
done
