set -e
mkdir -p gpurun_out/r1s6
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r1s6/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1s6/smoke.log 2>&1
timeout -k 10 240 python bench.py > gpurun_out/r1s6/bench_block.json 2> gpurun_out/r1s6/bench_block.err
timeout -k 10 240 python bench.py --workload sig > gpurun_out/r1s6/bench_sig.json 2> gpurun_out/r1s6/bench_sig.err
timeout -k 10 240 python bench.py --workload mvcc > gpurun_out/r1s6/bench_mvcc.json 2> gpurun_out/r1s6/bench_mvcc.err
timeout -k 10 300 python bench.py --workload c5 > gpurun_out/r1s6/bench_c5.json 2> gpurun_out/r1s6/bench_c5.err
echo all-done
