#!/bin/bash
# round 3: C4 with k_sha256 on a second stream beside k_der + k_inv (FGV_SIG_FORK A/B), crypto
# GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3ze
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_crypto.py tests/test_gpu_group.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for fk in 1 0; do
    FGV_SIG_FORK=$fk timeout -k 10 300 python -u bench.py --workload sig --steps 20 --warmup 3 --cpu-threads 0 > $O/sig_f${fk}_$rep.json 2> $O/sig_f${fk}_$rep.err || { echo sig failed; tail -20 $O/sig_f${fk}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/sig_f${fk}_$rep.json')); print('fork $fk rep $rep', d['value'], d['ms_per_step'], d.get('parity_vs_oracle', d.get('parity')))"
  done
done
echo done
