#!/bin/bash
# A/B of the pipelined committer's ahead placements (FGV_AHEAD), alternating runs on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for m in ${MODES:-0 4 2}; do
    FGV_AHEAD=$m timeout -k 10 240 python bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency \
      > gpurun_out/ab/ahead_${m}_$rep.json 2> gpurun_out/ab/ahead_${m}_$rep.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab/ahead_${m}_$rep.json'));print('mode $m rep $rep', d['value'], d['ms_per_step'])"
  done
done
