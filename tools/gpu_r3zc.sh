#!/bin/bash
# round 3: 2-rank rehearsal (gloo, one GPU) at HEAD and at the session-start build (_old/) with
# the mismatching transactions logged
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r3zc
mkdir -p $O
FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-pcie --no-latency --cpu-threads 0 > $O/head.json 2> $O/head.err || { echo head failed; tail -30 $O/head.err; exit 1; }
grep 'differ' $O/head.err | head -20
cd _old
FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 1 --no-pcie --no-latency --cpu-threads 0 > $O/old.json 2> $O/old.err || { echo old failed; tail -30 $O/old.err; exit 1; }
grep 'differ' $O/old.err | head -20
echo done
