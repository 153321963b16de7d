#!/bin/bash
# Kernel + memory-copy timeline traces of the block and mvcc workloads (no counters).
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/trace
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $OUT/block -o run -- python bench.py --steps 6 --warmup 2 --cpu-threads 0 > $OUT/block.json 2> $OUT/block.err
timeout -k 10 240 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $OUT/mvcc -o run -- python bench.py --workload mvcc --steps 6 --warmup 2 > $OUT/mvcc.json 2> $OUT/mvcc.err
echo trace-done
