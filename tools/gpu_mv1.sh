set -e
mkdir -p gpurun_out/r2_mv1
timeout -k 10 300 python -u -m pytest tests/test_gpu_mvcc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_mv1/gpu_tests.log 2>&1
timeout -k 10 200 python bench.py --workload mvcc > gpurun_out/r2_mv1/bench_mvcc.json 2> gpurun_out/r2_mv1/bench_mvcc.err
echo done
