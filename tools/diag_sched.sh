#!/bin/bash
# Throughput of graph scheduling variants (diagnostic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local tag="$1"; shift
  env "$@" timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --no-cpu-baseline --no-roofline \
      > gpurun_out/sched_$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/sched_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/sched_$tag.log)"
}
run base X=1
run nb2 SACX_NBATCH=2
run nb8 SACX_NBATCH=8
run nb8g64 SACX_NBATCH=8 SACX_GRAPH_STEPS=64
run nb1 SACX_NBATCH=1
run fuse SACX_FUSE=1
