#!/bin/bash
# round 3: k_mvx_extract with parallel LDS staging, transactions per workgroup A/B (FGV_MVX_TPW
# 16 / 32 / 64) on the chained C3 bench, MVCC GPU tests at the default, a trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
FGV_MVX_TPW=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py > $O/tests16.log 2>&1 || { echo tests16 failed; tail -60 $O/tests16.log; exit 1; }
tail -1 $O/tests16.log
for rep in 1 2; do
  for tp in 16 32 64; do
    FGV_MVX_TPW=$tp timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 --mvcc-single-steps 20 > $O/tp${tp}_$rep.json 2> $O/tp${tp}_$rep.err || { echo mvcc failed; tail -20 $O/tp${tp}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/tp${tp}_$rep.json')); print('tpw $tp rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
  done
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/t10 -o run -- python bench.py --workload mvcc --steps 20 --warmup 2 --mvcc-chain 10 --mvcc-single-steps 4 > $O/t10.json 2> $O/t10.err || { echo trace failed; tail -20 $O/t10.err; exit 1; }
echo done
