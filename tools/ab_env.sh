#!/bin/bash
# A/B of an environment knob over alternating bench runs on one box:
#   VAR=FGV_SHA_PRIO VALUES="1 2 3" REPS=2 bash tools/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for rep in $(seq 1 ${REPS:-2}); do
  for v in $VALUES; do
    env $VAR=$v timeout -k 10 240 python bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency $EXTRA \
      > gpurun_out/ab/${VAR}_${v}_$rep.json 2> gpurun_out/ab/${VAR}_${v}_$rep.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab/${VAR}_${v}_$rep.json'));print('$VAR=$v rep $rep', d['value'], d['ms_per_step'], d.get('kernel_ms'))"
  done
done
