#!/bin/bash
# round 3: key-level endorsement on the device fold: SBE GPU tests first, then the whole GPU
# suite, tools/bench_sbe.py, the default bench, and a clean block-step kernel profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sbe.py > $O/sbe.log 2>&1 || { echo sbe tests failed; tail -60 $O/sbe.log; exit 1; }
tail -2 $O/sbe.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/bench_sbe.py > $O/sbe.json 2> $O/sbe.err || { echo bench_sbe failed; tail -20 $O/sbe.err; exit 1; }
cat $O/sbe.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['kernel_ms'])"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats --kernel-exclude-regex "k_gtab|k_keytab" -d $O/blockprof -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/blockprof.json 2> $O/blockprof.err || { echo blockprof failed; tail -20 $O/blockprof.err; exit 1; }
echo done
