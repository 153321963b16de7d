#!/bin/bash
# Collects the rocprofv3 evidence committed under profiles/ (run on the GPU box via gpurun).
#   1. kernel trace + stats of the headline bench (block workload: 32-block steps only, no
#      single-block latency or PCIe passes) and of the sig / mvcc workloads
#   2. PMC passes (separate runs, --kernel-trace only): VALU instruction counts / busy cycles for
#      the crypto kernels, FETCH_SIZE / WRITE_SIZE for MVCC
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${PROF_OUT:-gpurun_out/prof}
mkdir -p $OUT
P="rocprofv3 --output-format csv"
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/block -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $OUT/block.json 2> $OUT/block.err
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/sig -o run -- python bench.py --workload sig --steps 10 --warmup 2 --cpu-threads 0 > $OUT/sig.json 2> $OUT/sig.err
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/mvcc -o run -- python bench.py --workload mvcc --steps 50 --warmup 3 > $OUT/mvcc.json 2> $OUT/mvcc.err
timeout -k 10 300 $P --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_valu -o run -- python bench.py --workload sig --steps 3 --warmup 1 --cpu-threads 0 > $OUT/pmc_valu.json 2> $OUT/pmc_valu.err
timeout -k 10 300 $P --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_fetch -o run -- python bench.py --workload mvcc --steps 10 --warmup 2 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err
timeout -k 10 300 $P --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python bench.py --workload mvcc --steps 10 --warmup 2 > $OUT/pmc_write.json 2> $OUT/pmc_write.err
timeout -k 10 300 $P --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_blk_valu -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $OUT/pmc_blk_valu.json 2> $OUT/pmc_blk_valu.err
timeout -k 10 300 $P --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_blk_fetch -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $OUT/pmc_blk_fetch.json 2> $OUT/pmc_blk_fetch.err
timeout -k 10 300 $P --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_blk_write -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $OUT/pmc_blk_write.json 2> $OUT/pmc_blk_write.err
timeout -k 10 300 $P --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/pmc_sig_fetch -o run -- python bench.py --workload sig --steps 3 --warmup 1 --cpu-threads 0 > $OUT/pmc_sig_fetch.json 2> $OUT/pmc_sig_fetch.err
timeout -k 10 300 $P --kernel-trace --pmc WRITE_SIZE -d $OUT/pmc_sig_write -o run -- python bench.py --workload sig --steps 3 --warmup 1 --cpu-threads 0 > $OUT/pmc_sig_write.json 2> $OUT/pmc_sig_write.err
# the cold-key path: C4 with every item its own key (k_vb_mul dominant)
timeout -k 10 300 $P --kernel-trace --stats -d $OUT/sigchurn -o run -- python bench.py --workload sig --sig-keys 131072 --steps 5 --warmup 1 --cpu-threads 0 > $OUT/sigchurn.json 2> $OUT/sigchurn.err
timeout -k 10 300 $P --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $OUT/pmc_sigchurn_valu -o run -- python bench.py --workload sig --sig-keys 131072 --steps 3 --warmup 1 --cpu-threads 0 > $OUT/pmc_sigchurn_valu.json 2> $OUT/pmc_sigchurn_valu.err
echo profile-done
