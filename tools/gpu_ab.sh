set -e
O=gpurun_out/ab2
mkdir -p $O
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 240 python bench.py --cpu-threads 0 > $O/bench_block.json 2> $O/bench_block.err
timeout -k 10 240 python bench.py --workload sig --cpu-threads 0 > $O/bench_sig.json 2> $O/bench_sig.err
echo all-done
