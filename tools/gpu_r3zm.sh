#!/bin/bash
# round 3: word-load hex decode of txid keys (k_fin_rows, k_fin_index_dev, k_bd_fold): the full
# GPU suite, C2 lean x3 (compare 0.655-0.696), a C2 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zm
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/lean_$rep.json 2> $O/lean_$rep.err || { echo lean failed; tail -20 $O/lean_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lean_$rep.json')); print('lean rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/st -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/st.json 2> $O/st.err || { echo trace failed; tail -20 $O/st.err; exit 1; }
echo done
