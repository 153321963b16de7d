#!/bin/bash
# round 3: C2 knob sweep on the current code (lean harness, 40 steps, alternating x2):
# FGV_AHEAD 2 (default) / 4, FGV_POINT_LANES auto / 2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3zk
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/$n.json 2> $O/$n.err || { echo $n failed; tail -20 $O/$n.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['parity_vs_labels'])"
}
for rep in 1 2; do
  run base_$rep FGV_AHEAD=2 || exit 1
  run ahead4_$rep FGV_AHEAD=4 || exit 1
  run lanes2_$rep FGV_POINT_LANES=2 || exit 1
done
echo done
