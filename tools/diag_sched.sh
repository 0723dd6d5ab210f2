#!/bin/bash
# Throughput of graph scheduling variants (diagnostic).
#   tools/diag_sched.sh [tag:VAR=val[,VAR=val...] ...]   (default: the sampler-batch sweep)
# BENCH_ARGS adds bench.py flags (e.g. "--config humanoid_eo").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag="$1"; shift
  env "$@" timeout -k 10 180 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-} \
      > gpurun_out/sched_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/sched_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/sched_$tag.log)"
}
if [ $# -eq 0 ]; then
  set -- base:X=1 nb2:SACX_NBATCH=2 nb8:SACX_NBATCH=8 nb8g64:SACX_NBATCH=8,SACX_GRAPH_STEPS=64 \
         nb1:SACX_NBATCH=1
fi
for v in "$@"; do
  tag="${v%%:*}"; vars="${v#*:}"
  run "$tag" ${vars//,/ } || exit 1
done
