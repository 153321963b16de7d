#!/bin/bash
# round 3: parse prefetch + MVCC one-walk/touch defaults: GPU tests, the default bench, MVCC
# over 100 blocks, bench_sbe (HBM-resident pipelined), then the round's rocprof evidence again
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['kernel'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['cpu_baseline']['value'], d['kernel_ms'])"
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mvcc.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
timeout -k 10 400 python -u tools/bench_sbe.py > $O/sbe.json 2> $O/sbe.err || { echo bench_sbe failed; tail -20 $O/sbe.err; exit 1; }
cat $O/sbe.json
for rep in 1 2; do
  for tv in 1 0; do
    FGV_FOLD_TOUCH=$tv timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/fold_t${tv}_$rep.json 2> $O/fold_t${tv}_$rep.err || { echo fold ab failed; tail -20 $O/fold_t${tv}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/fold_t${tv}_$rep.json')); print('fold touch $tv rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms']['k_bd_fold'])"
  done
done
PROF_OUT=$O/prof bash tools/profile_round.sh || { echo profile failed; exit 1; }
echo done
