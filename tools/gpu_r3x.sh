#!/bin/bash
# round 3: staging ring of three arenas + fgv_prefetch (batch k stages batch k+2): block GPU tests,
# the default bench (PCIe-inclusive pass), and a copy trace of that pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_blocks.py tests/test_gpu_shard_procs.py tests/test_gpu_group.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['pcie_inclusive'])"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $O/tp -o run -- python bench.py --steps 6 --warmup 2 --cpu-threads 0 --no-latency > $O/tp.json 2> $O/tp.err || { echo trace failed; tail -20 $O/tp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tp.json')); print(d['value'], d['ms_per_step'], d['pcie_inclusive'])"
echo done
