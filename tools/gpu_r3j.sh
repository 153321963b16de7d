#!/bin/bash
# round 3: the next batch's k_bd_emit / k_der / k_inv ahead with its front half (per-set verify
# buffers) and the verify chain queued before the early finalize: GPU tests, then alternating
# lean A/Bs of FGV_PREFIX_AHEAD and FGV_FOLD_TOUCH, then the default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for pv in 1 0; do
    FGV_PREFIX_AHEAD=$pv timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/prefix_${pv}_$rep.json 2> $O/prefix_${pv}_$rep.err || { echo prefix ab failed; tail -20 $O/prefix_${pv}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/prefix_${pv}_$rep.json')); print('prefix ahead $pv rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
  done
  FGV_FOLD_TOUCH=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/foldt_$rep.json 2> $O/foldt_$rep.err || { echo fold ab failed; tail -20 $O/foldt_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/foldt_$rep.json')); print('fold touch 1 rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['kernel'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['cpu_baseline']['value'], d['kernel_ms'])"
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mvcc.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
timeout -k 10 400 python -u tools/bench_sbe.py > $O/sbe.json 2> $O/sbe.err || { echo bench_sbe failed; tail -20 $O/sbe.err; exit 1; }
cat $O/sbe.json
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/trace -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/trace.json 2> $O/trace.err || { echo trace failed; tail -20 $O/trace.err; exit 1; }
echo done
