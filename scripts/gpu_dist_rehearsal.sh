#!/bin/bash
# Multi-rank rehearsal on a 1-GPU box: 2 ranks share cuda:0, gloo backend (RCCL needs one GPU per rank).
# Exercises bench.py's distributed path: parameter broadcast, per-step flat-bucket all-reduce after the
# graph replay, optimizer, metric sync, barriers, max-over-ranks timing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MTA_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 5 > gpurun_out/dist2.json 2> gpurun_out/dist2.err
