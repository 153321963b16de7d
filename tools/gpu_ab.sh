set -e
O=gpurun_out/ab3
mkdir -p $O
for i in 1 2; do
timeout -k 10 240 python bench.py --cpu-threads 0 > $O/bench_block_$i.json 2> $O/bench_block_$i.err
done
timeout -k 10 240 python bench.py --workload c5 --cpu-threads 0 > $O/bench_c5.json 2> $O/bench_c5.err
echo all-done
