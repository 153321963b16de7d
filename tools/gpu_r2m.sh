#!/bin/bash
# device-side verify counts + fused single-GPU call: block tests, then the block bench + a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_blocks.py tests/test_gpu_crypto.py tests/test_gpu_blocksig.py tests/test_gpu_known_answers.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u bench.py --cpu-threads 0 > $O/bench_block.json 2> $O/bench_block.err || { echo bench failed; tail -30 $O/bench_block.err; exit 1; }
cat $O/bench_block.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms'], d['host_ms'], d['latency_1block_ms'], (d['pcie_inclusive'] or {}).get('value'))"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/prof_block -o run -- python3 bench.py --cpu-threads 0 --no-pcie --no-latency --steps 12 > $O/prof_block.json 2> $O/prof_block.err || { echo prof failed; tail -5 $O/prof_block.err; exit 1; }
echo done
