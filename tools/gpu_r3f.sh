#!/bin/bash
# round 3: coalesced H2D copies + one-wave k_bd_sha default: GPU tests, default bench, then the
# round's rocprofv3 evidence (tools/profile_round.sh: kernel stats + separate PMC passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['frac'], d['pcie_inclusive'], d['kernel_ms'])"
PROF_OUT=$O/prof bash tools/profile_round.sh || { echo profile failed; exit 1; }
echo done
