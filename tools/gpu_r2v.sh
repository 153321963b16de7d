#!/bin/bash
# round-2 refresh, part 2: rocprof kernel traces and PMC passes (tools/profile_round.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2v
mkdir -p $O
timeout -k 10 1100 bash tools/profile_round.sh > $O/profile.log 2>&1 || { echo profile failed; tail -20 $O/profile.log; exit 1; }
tail -1 $O/profile.log
timeout -k 10 400 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/bench_mvcc100.json 2> $O/bench_mvcc100.err || { echo bench mvcc failed; tail -20 $O/bench_mvcc100.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mvcc100.json')); print('mvcc100', d['value'], d['ms_per_step'])"
echo done
