#!/bin/bash
# round 3: X.509 / PEM fork-hazard rules, key-level batch rule, GPU tests + one default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 20 > $O/b1.json 2> $O/b1.err || { echo bench failed; tail -20 $O/b1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/b1.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'])"
echo done
