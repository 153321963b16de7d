#!/bin/bash
# round 3: chained MVCC with block 0 enqueued before the other heads and pre-bound ctypes
# arguments (tests, C3 bench), then the round's evidence (tools/gpu_r3z.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3za
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mvcc.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
bash tools/gpu_r3z.sh
