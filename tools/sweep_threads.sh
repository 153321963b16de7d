# A/B of the engine's host worker count (FGV_HOST_THREADS) on the C3 and C2 benches
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-threads}
mkdir -p $O
nproc > $O/nproc.txt
for t in ${THREADS:-4 8 12 16 24}; do
  FGV_HOST_THREADS=$t timeout -k 10 120 python bench.py --workload mvcc --cpu-threads 0 > $O/mvcc_t$t.json 2> $O/mvcc_t$t.err
  FGV_HOST_THREADS=$t timeout -k 10 120 python bench.py --cpu-threads 0 > $O/block_t$t.json 2> $O/block_t$t.err
done
echo sweep-done
