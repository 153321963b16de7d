#!/bin/bash
# round 3: k_mvx_extract with load-batched LDS staging and record copies: MVCC GPU tests, C3
# chained bench x2, kernel stats of the chained run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zf
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc_$rep.json 2> $O/mvcc_$rep.err || { echo mvcc failed; tail -20 $O/mvcc_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/mvcc_$rep.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/st -o run -- python bench.py --workload mvcc --steps 50 --warmup 3 > $O/st.json 2> $O/st.err || { echo stats failed; tail -20 $O/st.err; exit 1; }
grep -i 'extract\|Name' $O/st/run_kernel_stats.csv | head -5
echo done
