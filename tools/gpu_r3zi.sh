#!/bin/bash
# round 3 final check at HEAD: smoke(), the full GPU suite, the default bench, C3 / C4 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zi
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('frac_profiled'), d['pcie_inclusive']['ms_per_step'], d['latency_1block_ms'])"
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mvcc.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
timeout -k 10 300 python -u bench.py --workload sig --steps 20 --warmup 3 > $O/sig.json 2> $O/sig.err || { echo sig failed; tail -20 $O/sig.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/sig.json')); print('sig', d['value'], d['ms_per_step'])"
echo done
