#!/bin/bash
# round 3: defaults after the A/Bs (prefix ahead off, MVCC polled wait, no memset): GPU tests of
# the touched paths, MVCC spin A/B over 100 blocks, the default bench, then the round's rocprof
# evidence (tools/profile_round.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py tests/test_gpu_sbe.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sv in 1 0; do
  FGV_MVCC_SPIN=$sv timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc_spin$sv.json 2> $O/mvcc_spin$sv.err || { echo mvcc failed; tail -20 $O/mvcc_spin$sv.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/mvcc_spin$sv.json')); print('mvcc spin $sv', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['kernel'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['cpu_baseline']['value'], d['kernel_ms'])"
PROF_OUT=$O/prof bash tools/profile_round.sh || { echo profile failed; exit 1; }
echo done
