#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O
export FGV_AHEAD=0
B="python3 bench.py --cpu-threads 0 --no-latency --no-pcie --steps 4 --warmup 1 --batches 2"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $O/p2 -o run -- $B > $O/p2.json 2> $O/p2.err || { echo p2 failed; tail -5 $O/p2.err; exit 1; }
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE -d $O/p3 -o run -- $B > $O/p3.json 2> $O/p3.err || { echo p3 failed; tail -5 $O/p3.err; }
echo done
