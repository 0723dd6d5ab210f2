#!/bin/bash
# bench.py's multi-process path on a one-GPU box: 2 ranks share GPU 0 over gloo.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
SACX_SHARE_DEVICE=1 SACX_REPLICA_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 50 \
  --no-cpu-baseline > gpurun_out/multi.log 2>&1
rc=$?; grep '^{' gpurun_out/multi.log | cut -c1-400; tail -3 gpurun_out/multi.log; exit $rc
