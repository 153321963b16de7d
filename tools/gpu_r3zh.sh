#!/bin/bash
# round 3: finalize front at wave priority 3 (FGV_FIN_PRIO 1 vs 0, C2 lean harness, alternating
# x3), committer GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zh
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_known_answers.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for fp in 1 0; do
    FGV_FIN_PRIO=$fp timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/fp${fp}_$rep.json 2> $O/fp${fp}_$rep.err || { echo lean failed; tail -20 $O/fp${fp}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/fp${fp}_$rep.json')); print('fin prio $fp rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
  done
done
echo done
