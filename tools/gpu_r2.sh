# round-2 GPU check: tests, smoke, bench lines.  usage: bash tools/gpu_r2.sh OUTDIR [bench workloads...]
set -e
OUT=${1:-gpurun_out/r2}
shift || true
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for w in "${@:-block}"; do
  timeout -k 10 300 python bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err
done
echo all-done
