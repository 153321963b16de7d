#!/bin/bash
# round 3: two-wave k_bd_sha2 + live k_point28 events: GPU tests, default bench, A/B of the
# split, and a kernel + memory-copy trace of the PCIe-inclusive (pinned) pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['kernel_ms'])"
for rep in 1 2; do
  for sp in 1 0; do
    FGV_SHA_SPLIT=$sp timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/ab_split${sp}_$rep.json 2> $O/ab_split${sp}_$rep.err || { echo ab failed; tail -20 $O/ab_split${sp}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ab_split${sp}_$rep.json')); print('split $sp rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms']['k_bd_sha'])"
  done
done
timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace --stats -d $O/copytrace -o run -- python bench.py --steps 12 --warmup 2 --cpu-threads 0 --no-latency > $O/copytrace.json 2> $O/copytrace.err || { echo trace failed; tail -20 $O/copytrace.err; exit 1; }
echo done
