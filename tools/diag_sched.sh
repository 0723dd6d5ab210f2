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
run nomerge SACX_MERGE_ALPHA=0
run g64 SACX_GRAPH_STEPS=64
run nofuse SACX_FUSE=0
