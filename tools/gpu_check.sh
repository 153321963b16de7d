# GPU tests + C2 bench + C2 kernel stats (one gpurun call); every step time-limited, chained by set -e
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 240 python bench.py > $O/bench_block.json 2> $O/bench_block.err
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/block -o run -- python bench.py --steps 10 --warmup 2 --cpu-threads 0 > $O/block_prof.json 2> $O/block_prof.err
echo check-done
