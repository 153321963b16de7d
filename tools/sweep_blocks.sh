#!/bin/bash
# C2 throughput / latency vs batch depth (blocks of 500 tx per validation pass), 1 GPU.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/sweep
mkdir -p $O
for b in 1 4 8 16 32 64; do
  timeout -k 10 240 python bench.py --blocks-per-gpu $b --cpu-threads 0 > $O/block_b$b.json 2> $O/block_b$b.err
done
echo sweep-done
