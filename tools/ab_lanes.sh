# A/B of k_point lanes per verify (FGV_POINT_LANES; "" = automatic choice)
set -e
for L in "" 1 2 3 4; do
  FGV_POINT_LANES=$L timeout -k 10 200 python bench.py --cpu-threads 0 --steps 20 > gpurun_out/b$L.json 2>/dev/null
  FGV_POINT_LANES=$L timeout -k 10 200 python bench.py --workload sig --cpu-threads 0 --steps 20 > gpurun_out/s$L.json 2>/dev/null
  python -c "import json; d=json.load(open('gpurun_out/b$L.json')); s=json.load(open('gpurun_out/s$L.json')); print('L=$L block', d['value'], d['stage_ms'], 'sig', s['value'], s['stage_ms'], s['parity_vs_labels'], d['parity_vs_labels'])"
done
