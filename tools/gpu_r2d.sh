#!/bin/bash
# point-kernel queue + pipelining: crypto/blocks tests, bench A/B (ahead on/off)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_crypto.py tests/test_gpu_blocks.py > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --cpu-threads 0 --no-latency > $O/bench_ahead.json 2> $O/bench_ahead.err || { echo bench failed; tail -30 $O/bench_ahead.err; exit 1; }
FGV_AHEAD=0 timeout -k 10 300 python -u bench.py --cpu-threads 0 --no-latency --no-pcie > $O/bench_noahead.json 2> $O/bench_noahead.err || { echo bench2 failed; tail -30 $O/bench_noahead.err; exit 1; }
python3 - <<'PY'
import json
for f in ("ahead", "noahead"):
    d = json.load(open(f"gpurun_out/r2d/bench_{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["parity_vs_labels"], (d.get("pcie_inclusive") or {}).get("value"), d["kernel_ms"])
PY
