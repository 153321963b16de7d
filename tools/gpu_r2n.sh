#!/bin/bash
# front chain on the main stream, joined digest event: block tests, bench per ahead mode, trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_blocks.py tests/test_gpu_known_answers.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 0 2; do
  FGV_AHEAD=$m timeout -k 10 300 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 30 > $O/bench_a$m.json 2> $O/bench_a$m.err || { echo bench $m failed; tail -30 $O/bench_a$m.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_a$m.json')); print('ahead $m', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms'])"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/prof_block -o run -- python3 bench.py --cpu-threads 0 --no-pcie --no-latency --steps 12 > $O/prof_block.json 2> $O/prof_block.err || { echo prof failed; tail -5 $O/prof_block.err; exit 1; }
echo done
