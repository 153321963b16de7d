#!/bin/bash
# round 3: kernel timelines of the C3 bench, chained (10 blocks per call) and one call per block
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
for ch in 10 1; do
  timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $O/t$ch -o run -- python bench.py --workload mvcc --steps 20 --warmup 2 --mvcc-chain $ch --mvcc-single-steps 4 > $O/t$ch.json 2> $O/t$ch.err || { echo trace failed; tail -20 $O/t$ch.err; exit 1; }
done
find $O -name '*.csv' | head
echo done
