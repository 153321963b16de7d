#!/bin/bash
# after moving the batch counters' D2H behind the finalize and dropping the parse prefetch knob
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 20 > $O/b$rep.json 2> $O/b$rep.err || { echo bench failed; tail -20 $O/b$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$rep.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'])"
done
echo done
