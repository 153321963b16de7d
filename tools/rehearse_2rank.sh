#!/bin/bash
# Multi-rank bench rehearsal on ONE GPU: 2 ranks over gloo sharing cuda:0 (the driver runs the
# real N=2..8 over RCCL on an 8-GPU node).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearse
FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/rehearse/block_2rank.json 2> gpurun_out/rehearse/block_2rank.err
echo rehearse-done
