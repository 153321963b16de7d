#!/bin/bash
# round-2 refresh: full GPU suite, smoke, the bench of every workload (profiles: gpu_r2v.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_block.json 2> $O/bench_block.err || { echo bench failed; tail -30 $O/bench_block.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_block.json')); print('C2', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['latency_1block_ms'], d['pcie_inclusive']['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
for w in sig mvcc c5; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo bench $w failed; tail -30 $O/bench_$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'])"
done
echo done
