#!/bin/bash
# key-level parameters through the MVCC commit, the committer suites (early finalize index), and
# A/Bs of the parse prefetch and the early finalize
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sbe.py tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py tests/test_gpu_blocks.py tests/test_gpu_known_answers.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_parse_pf.sh > $O/ab_pf.log 2>&1 || { echo ab failed; tail -20 $O/ab_pf.log; exit 1; }
cat $O/ab_pf.log
echo done
