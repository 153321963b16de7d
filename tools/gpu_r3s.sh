#!/bin/bash
# round 3: C2 A/B of k_bd_parse lanes per workgroup (FGV_PARSE_LANES 16 / 32 / 64, lean harness,
# alternating), then a kernel trace of the default C2 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_blocks.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for pl in 16 32 64; do
    FGV_PARSE_LANES=$pl timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/pl${pl}_$rep.json 2> $O/pl${pl}_$rep.err || { echo ab failed; tail -20 $O/pl${pl}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/pl${pl}_$rep.json')); print('parse lanes $pl rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms']['k_bd_parse'])"
  done
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace -d $O/tc2 -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/tc2.json 2> $O/tc2.err || { echo trace failed; tail -20 $O/tc2.err; exit 1; }
echo done
