set -e
O=gpurun_out/ab9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
timeout -k 10 240 python bench.py --workload mvcc > $O/bench_mvcc_$i.json 2> $O/bench_mvcc_$i.err
done
timeout -k 10 240 python bench.py --workload mvcc --no-presplit > $O/bench_mvcc_nopre.json 2> $O/bench_mvcc_nopre.err
echo all-done
