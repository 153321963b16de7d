#!/bin/bash
# full GPU suite + every bench workload + rocprofv3 kernel stats (round-2 evidence)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench_block.json 2> $O/bench_block.err || { echo bench block failed; tail -30 $O/bench_block.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload sig > $O/bench_sig.json 2> $O/bench_sig.err || { echo bench sig failed; tail -30 $O/bench_sig.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/bench_mvcc.json 2> $O/bench_mvcc.err || { echo bench mvcc failed; tail -30 $O/bench_mvcc.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c5 --cpu-threads 0 --no-latency > $O/bench_c5.json 2> $O/bench_c5.err || { echo bench c5 failed; tail -30 $O/bench_c5.err; exit 1; }
P="rocprofv3 --output-format csv --kernel-trace --stats"
timeout -k 10 300 $P -d $O/prof_block -o run -- python3 bench.py --cpu-threads 0 --no-pcie --no-latency --steps 12 > $O/prof_block.json 2> $O/prof_block.err || { echo prof block failed; tail -5 $O/prof_block.err; exit 1; }
timeout -k 10 300 $P -d $O/prof_sig -o run -- python3 bench.py --workload sig --cpu-threads 0 --steps 10 > $O/prof_sig.json 2> $O/prof_sig.err || { echo prof sig failed; exit 1; }
timeout -k 10 300 $P -d $O/prof_mvcc -o run -- python3 bench.py --workload mvcc --steps 100 --warmup 5 > $O/prof_mvcc.json 2> $O/prof_mvcc.err || { echo prof mvcc failed; exit 1; }
for w in block sig mvcc c5; do python3 -c "import json,sys; d=json.load(open('$O/bench_$w.json')); print('$w', d['value'], d['unit'], d['ms_per_step'], d.get('parity_vs_labels'), (d.get('pcie_inclusive') or {}).get('value'), d.get('latency_1block_ms'), d['roofline'].get('frac'))"; done
