#!/bin/bash
# round 3: multi-rank rehearsal of the default bench (2 ranks over gloo on the one GPU) and the
# C5 workload record
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zb
mkdir -p $O
FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $O/block_2rank.json 2> $O/block_2rank.err || { echo rehearsal failed; tail -30 $O/block_2rank.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/block_2rank.json')); print('2rank', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['n_gpus'], d['config'].get('parallelism'))"
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 1 > $O/c5.json 2> $O/c5.err || { echo c5 failed; tail -20 $O/c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c5.json')); print('c5', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
echo done
