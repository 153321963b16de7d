# GPU tests + C3 bench (public and with private data) in one gpurun call
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-check2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 240 python bench.py --workload mvcc > $O/bench_mvcc.json 2> $O/bench_mvcc.err
timeout -k 10 240 python bench.py --workload mvcc --mvcc-private-every 8 > $O/bench_mvcc_private.json 2> $O/bench_mvcc_private.err
echo check2-done
