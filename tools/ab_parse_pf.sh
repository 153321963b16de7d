#!/bin/bash
# A/B: k_bd_parse prefetch of each envelope's first N bytes (FGV_PARSE_PF), alternating runs
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab_pf
mkdir -p $O
for rep in 1 2; do
  for pf in 0 1024 4096 8192; do
    FGV_PARSE_PF=$pf timeout -k 10 200 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 20 > $O/pf${pf}_$rep.json 2> $O/pf${pf}_$rep.err || { echo bench failed; tail -20 $O/pf${pf}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/pf${pf}_$rep.json')); kt=d.get('kernel_ms') or {}; print('pf=$pf', d['ms_per_step'], d['parity_vs_labels'], kt.get('k_bd_parse', kt))"
  done
done
