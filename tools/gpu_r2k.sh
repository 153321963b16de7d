#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rangequery.py tests/test_gpu_mvcc.py tests/test_gpu_ledgers.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
