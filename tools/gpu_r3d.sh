#!/bin/bash
# round 3: 13-bit key comb + one-reduction y3, principals, default ahead: GPU tests, default
# bench, kernel-trace stats of 32-block steps, one VALU PMC pass
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo tests failed; tail -80 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 20 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['frac'], d['kernel_ms'])"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/prof -o run -- python bench.py --steps 20 --warmup 2 --cpu-threads 0 --no-pcie --no-latency > $O/prof.json 2> $O/prof.err || { echo prof failed; tail -20 $O/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_valu -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $O/pmc_valu.json 2> $O/pmc_valu.err || { echo pmc failed; tail -20 $O/pmc_valu.err; exit 1; }
echo done
