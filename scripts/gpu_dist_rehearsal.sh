#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: 2 ranks share cuda:0 over gloo (RCCL needs one GPU per
# rank); exercises sharding, the gradient all-reduce, max-over-ranks timing and the JSON line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export VISSM_DIST_BACKEND=gloo
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 2 --warmup 1 --B 8192 > gpurun_out/dist2.log 2>&1
rc=$?; tail -3 gpurun_out/dist2.log | cut -c1-600; exit $rc
