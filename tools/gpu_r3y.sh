#!/bin/bash
# round 3: k_bd_count with one atomic per workgroup and kind: committer GPU tests, C2 lean x3,
# a C2 kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_known_answers.py tests/test_gpu_channel.py tests/test_gpu_sbe.py tests/test_gpu_group.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/lean_$rep.json 2> $O/lean_$rep.err || { echo lean failed; tail -20 $O/lean_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/lean_$rep.json')); print('lean rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/tc2 -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/tc2.json 2> $O/tc2.err || { echo trace failed; tail -20 $O/tc2.err; exit 1; }
echo done
