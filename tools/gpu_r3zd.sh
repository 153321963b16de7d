#!/bin/bash
# round 3: multi-rank rehearsals of the default bench over gloo on the one GPU (2 and 4 ranks)
# after the generator's label fix (a block's first tx drawn as a duplicate is unique)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zd
mkdir -p $O
for n in 2 4; do
  FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 5 --warmup 1 --cpu-threads 0 > $O/block_${n}rank.json 2> $O/block_${n}rank.err || { echo rehearsal $n failed; tail -30 $O/block_${n}rank.err; exit 1; }
  grep 'differ' $O/block_${n}rank.err | head -5
  python3 -c "import json; d=json.load(open('$O/block_${n}rank.json').read().split(chr(10))[-2] if False else open('$O/block_${n}rank.json')); print('${n}rank', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['pcie_inclusive']['parity_vs_labels'])" 2>/dev/null || tail -c 600 $O/block_${n}rank.json
done
echo done
