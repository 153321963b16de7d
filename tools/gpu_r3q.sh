#!/bin/bash
# round 3: chained MVCC with the framing walks on the host pool and zero-copy tails: tests, the
# C3 bench A/B (zero-copy on / off, one call per block), a kernel trace of the chained run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc_chain.py tests/test_gpu_mvcc.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "10 1" "1 1"; do
  set -- $v
  FGV_MVCC_ZC=$2 timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 --mvcc-chain $1 > $O/mvcc_c$1_z$2.json 2> $O/mvcc_c$1_z$2.err || { echo mvcc failed; tail -20 $O/mvcc_c$1_z$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/mvcc_c$1_z$2.json')); print('mvcc chain $1 zc $2', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/t10 -o run -- python bench.py --workload mvcc --steps 20 --warmup 2 --mvcc-chain 10 --mvcc-single-steps 4 > $O/t10.json 2> $O/t10.err || { echo trace failed; tail -20 $O/t10.err; exit 1; }
echo done
