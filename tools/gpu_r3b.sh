#!/bin/bash
# round 3: GPU tests, then the FGV_AHEAD=2 harness question: default bench vs A/B flags
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -k 10 400 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$n.json')); print('$n', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms'].get('k_bd_sha_payload'), d['kernel_ms'].get('k_point28'))"
}
run a0_full FGV_AHEAD=0 --steps 20
run a2_full FGV_AHEAD=2 --steps 20
run a2_lean20 FGV_AHEAD=2 --steps 20 --cpu-threads 0 --no-pcie --no-latency
run a2_lean60 FGV_AHEAD=2 --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency
run a0_lean60 FGV_AHEAD=0 --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency
echo done
