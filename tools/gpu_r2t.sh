#!/bin/bash
# committer suites after the fused fold+codes step and the parallel identity occurrences, then
# A/B of the early finalize (FGV_EARLY_FIN) at the new defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_blocks.py tests/test_gpu_known_answers.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do
  for ef in 1 0; do
    FGV_EARLY_FIN=$ef timeout -k 10 200 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 20 > $O/ef${ef}_$rep.json 2> $O/ef${ef}_$rep.err || { echo bench failed; tail -20 $O/ef${ef}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/ef${ef}_$rep.json')); k=d.get('kernel_ms') or {}; print('early_fin=$ef', d['ms_per_step'], d['parity_vs_labels'], {a: round(b, 4) for a, b in k.items()})"
  done
done
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/prof_block -o run -- python3 bench.py --cpu-threads 0 --no-pcie --no-latency --steps 12 > $O/prof_block.json 2> $O/prof_block.err || { echo prof failed; tail -5 $O/prof_block.err; exit 1; }
echo done
