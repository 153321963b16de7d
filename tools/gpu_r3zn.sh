#!/bin/bash
# round 3 last check: smoke() and the default bench (40 timed steps) at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zn
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline'].get('frac_profiled'), d['pcie_inclusive']['ms_per_step'], d['pcie_inclusive']['parity_vs_labels'], d['latency_1block_ms'], d['cpu_baseline']['value'])"
echo done
