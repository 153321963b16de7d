#!/bin/bash
# round 3: the default bench's timed-step count (10 vs 40 steps, alternating x2)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zj
mkdir -p $O
for rep in 1 2; do
  for st in 10 40; do
    timeout -k 10 400 python -u bench.py --steps $st --warmup 5 --no-latency > $O/s${st}_$rep.json 2> $O/s${st}_$rep.err || { echo bench failed; tail -20 $O/s${st}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s${st}_$rep.json')); print('steps $st rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
  done
done
echo done
