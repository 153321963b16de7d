#!/bin/bash
# round 3: fgv_mvcc_validate_blocks (consecutive blocks as one device chain): MVCC GPU tests, then
# the C3 bench chained (10 blocks per call) and one call per block
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for ch in 10 1; do
  timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 --mvcc-chain $ch > $O/mvcc_c$ch.json 2> $O/mvcc_c$ch.err || { echo mvcc failed; tail -20 $O/mvcc_c$ch.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/mvcc_c$ch.json')); print('mvcc chain $ch', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'], d['fixpoint_rounds'][:5])"
done
echo done
