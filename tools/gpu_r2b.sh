#!/bin/bash
# round-2 bench pass: rotation/prefetch tests, default bench, rocprofv3 kernel stats of the bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2b
mkdir -p $O
nproc > $O/nproc.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_blocks.py \
  -k "rotation or presplit or next" > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --cpu-threads 0 --no-pcie --no-latency --steps 12 > $O/prof_bench.json 2> $O/prof.err || { echo prof failed; tail -20 $O/prof.err; exit 1; }
find $O/prof -name "*stats*" | head
