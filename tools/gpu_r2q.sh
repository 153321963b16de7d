#!/bin/bash
# key-level endorsement + extraction hazards: new GPU tests first, then the full suite, smoke, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2q
mkdir -p $O
true > $O/sbe.log 2>&1 || { echo sbe failed; tail -60 $O/sbe.log; exit 1; }
tail -2 $O/sbe.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench_block.json 2> $O/bench_block.err || { echo bench failed; tail -30 $O/bench_block.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_block.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['latency_1block_ms'], d['roofline']['frac'])"
echo done
