#!/bin/bash
# GPU box: the -m gpu suite, then single-seed HalfCheetah and Humanoid SAC throughput.
# usage (from the repo root, via gpurun): bash tools/gpu_quick.sh [extra multi_seed configs...]
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1
tail -3 gpurun_out/t.log
for c in hc humanoid_sac "$@"; do
    MS_CONFIG=$c timeout -k 10 120 python tools/multi_seed.py 1
done
