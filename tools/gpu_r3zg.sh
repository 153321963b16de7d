#!/bin/bash
# round 3: chained extractions over two streams (FGV_MVX_STREAMS 2 vs 1, alternating): MVCC
# GPU tests, C3 chained bench x2 each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zg
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for xs in 2 1; do
    FGV_MVX_STREAMS=$xs timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/xs${xs}_$rep.json 2> $O/xs${xs}_$rep.err || { echo mvcc failed; tail -20 $O/xs${xs}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/xs${xs}_$rep.json')); print('streams $xs rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
  done
done
echo done
