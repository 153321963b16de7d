#!/bin/bash
# A/B, alternating runs (round 2, kept as the record of profiles/round2_ab/): k_bd_parse prefetch of each
# envelope's first N bytes (FGV_PARSE_PF, measured no gain and removed from the kernel) and
# the finalize's txid index beside the verify chain (FGV_EARLY_FIN)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/ab_pf
mkdir -p $O
for rep in 1 2; do
  for cfg in "0 1" "0 0" "4096 1" "1024 1"; do
    set -- $cfg
    FGV_PARSE_PF=$1 FGV_EARLY_FIN=$2 timeout -k 10 200 python -u bench.py --cpu-threads 0 --no-pcie --no-latency --steps 20 > $O/pf$1_ef$2_$rep.json 2> $O/pf$1_ef$2_$rep.err || { echo bench failed; tail -20 $O/pf$1_ef$2_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/pf$1_ef$2_$rep.json')); k=d.get('kernel_ms') or {}; print('pf=$1 early_fin=$2', d['ms_per_step'], d['parity_vs_labels'], round(k.get('k_bd_parse', 0), 4), round(k.get('batch', 0), 4))"
  done
done
