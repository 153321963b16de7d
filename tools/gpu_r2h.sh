#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
true
tail -2 $O/tests.log
for a in 3 0 2; do
FGV_AHEAD=$a timeout -k 10 300 python -u bench.py --cpu-threads 0 --no-latency --no-pcie > $O/bench_$a.json 2> $O/bench_$a.err || { echo bench failed; tail -30 $O/bench_$a.err; exit 1; }
done
python3 - <<'PY'
import json
for f in ("3", "0", "2"):
    d = json.load(open(f"gpurun_out/r2h/bench_{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["parity_vs_labels"], d["kernel_ms"], d["host_ms"])
PY
