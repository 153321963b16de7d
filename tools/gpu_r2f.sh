#!/bin/bash
# PMC passes on the device-parse committer kernels (FGV_AHEAD=0: kernels in isolation)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
export FGV_AHEAD=0
B="python3 bench.py --cpu-threads 0 --no-latency --no-pcie --steps 4 --warmup 1 --batches 2"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/kt -o run -- $B > $O/kt.json 2> $O/kt.err || { echo kt failed; tail -5 $O/kt.err; exit 1; }
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $O/p1 -o run -- $B > $O/p1.json 2> $O/p1.err || { echo p1 failed; tail -5 $O/p1.err; exit 1; }
grep -E "SQ_WAIT_INST_ANY|SQ_INSTS_VMEM_RD|SQ_INST_CYCLES_VMEM|SQ_WAIT_ANY|SQ_INSTS_FLAT|TA_BUSY|TCP_TCC_READ_REQ" $O/avail.txt | head -20 > $O/cands.txt || true
echo done
