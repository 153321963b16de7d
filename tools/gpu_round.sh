#!/bin/bash
# One GPU-box run (via gpurun) of named steps, each under its own time limit, stopping at the
# first failure:
#   bash tools/gpu_round.sh <out-name> <step> [<step> ...]
# Steps:
#   tests            the full GPU suite (pytest -m gpu)
#   tests:<expr>     GPU tests matching a -k expression
#   smoke            __graft_entry__.smoke()
#   bench            the default bench (C2 headline line)
#   lean<N>          N lean C2 runs (40 steps, no CPU baseline / PCIe / latency passes)
#   env:VAR=VAL:N    N lean C2 runs with an environment knob set (A/B)
#   shardp           C2 through the N>1 shard protocol at N=1 (lean)
#   leanx:<args>:N   N lean C2 runs with extra bench arguments (commas for spaces)
#   churn            C2 with every creator a distinct identity (the cold-key path)
#   sigchurn         C4 with every item its own key (registered cold)
#   churntrace       rocprofv3 kernel + HIP API trace of a short churn run
#   notorch | notorch2   the C2 line through the C ABI alone (no torch), one / two contexts
#   pipeline         the end-to-end commit pipeline (committer -> MVCC -> commit hash)
#   mvcc | sig | c5 | sbe   the other workloads (tools/bench_sbe.py for sbe)
#   mvccpmc          FETCH_SIZE / WRITE_SIZE passes of the mvcc workload
#   fetchcalib       FETCH_SIZE against known bytes (streaming read, random 64 B gathers)
#   trace            rocprofv3 --kernel-trace --stats of a C2 run
#   apitrace         kernel + HIP API trace of a C2 run (host enqueue costs)
#   lattrace         the same of tools/latency_probe.py (single-block calls)
#   profileblock     the block workload's part of it only
#   profile          tools/profile_round.sh (stats + PMC passes of every workload)
#   py:<file>        python <file> (a micro-benchmark or check under tools/)
#   with:VAR=VAL:<step>  <step> with VAR=VAL in its environment
# Output: gpurun_out/<out-name>/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
[ $# -ge 2 ] || { echo "usage: $0 <out-name> <step>..."; exit 2; }
O=gpurun_out/$1
shift
mkdir -p "$O"
show() { python3 -c "import json,sys; d=json.load(open('$1')); print('$2', *[d.get(k) for k in sys.argv[1:]])" "${@:3}"; }
for step in "$@"; do
  case "$step" in
    tests)
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 \
        || { echo tests failed; tail -60 $O/tests.log; exit 1; }
      tail -1 $O/tests.log ;;
    tests:*)
      k=${step#tests:}
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests -k "$k" > $O/tests_k.log 2>&1 \
        || { echo tests failed; tail -60 $O/tests_k.log; exit 1; }
      tail -1 $O/tests_k.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
        || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
      show $O/bench.json bench value ms_per_step parity_vs_labels latency_1block_ms
      python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('roofline', r['kernel'], r['frac'], r.get('frac_profiled'), 'pcie', d['pcie_inclusive']['ms_per_step'], 'cpu', d['cpu_baseline']['value'])" ;;
    leanx:*)
      # leanx:<bench args, commas for spaces>:N -- N lean C2 runs with extra bench arguments (A/B)
      spec=${step#leanx:}; n=${spec##*:}; xa=$(echo ${spec%:*} | tr ',' ' '); tag=$(echo ${spec%:*} | tr -c 'a-zA-Z0-9\n' '_')
      for rep in $(seq 1 $n); do
        timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency $xa > $O/leanx_${tag}_$rep.json 2> $O/leanx_${tag}_$rep.err \
          || { echo leanx $xa failed; tail -20 $O/leanx_${tag}_$rep.err; exit 1; }
        show $O/leanx_${tag}_$rep.json "lean $xa $rep" value ms_per_step parity_vs_labels
      done ;;
    lean*)
      n=${step#lean}; n=${n:-1}
      for rep in $(seq 1 $n); do
        timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/lean_$rep.json 2> $O/lean_$rep.err \
          || { echo lean failed; tail -20 $O/lean_$rep.err; exit 1; }
        show $O/lean_$rep.json "lean $rep" value ms_per_step parity_vs_labels
      done ;;
    env:*)
      # env:VAR=VAL:N -- N lean C2 runs with VAR=VAL (A/B against lean<N> on the same box)
      spec=${step#env:}; n=${spec##*:}; kv=${spec%:*}; tag=$(echo $kv | tr '= ' '__')
      for rep in $(seq 1 $n); do
        env $kv timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/lean_${tag}_$rep.json 2> $O/lean_${tag}_$rep.err \
          || { echo lean $kv failed; tail -20 $O/lean_${tag}_$rep.err; exit 1; }
        show $O/lean_${tag}_$rep.json "lean $kv $rep" value ms_per_step parity_vs_labels
      done ;;
    shardp)
      timeout -k 10 300 python -u bench.py --shard-protocol --steps 40 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/shardp.json 2> $O/shardp.err \
        || { echo shardp failed; tail -20 $O/shardp.err; exit 1; }
      show $O/shardp.json shardp value ms_per_step parity_vs_labels ;;
    churn)
      timeout -k 10 400 python -u bench.py --clients 16000 --steps 20 --warmup 3 --cpu-threads 0 --no-pcie > $O/churn.json 2> $O/churn.err \
        || { echo churn failed; tail -20 $O/churn.err; exit 1; }
      show $O/churn.json churn value ms_per_step parity_vs_labels latency_1block_ms ;;
    sigchurn)
      timeout -k 10 400 python -u bench.py --workload sig --sig-keys 131072 --steps 10 --warmup 2 --cpu-threads 0 > $O/sigchurn.json 2> $O/sigchurn.err \
        || { echo sigchurn failed; tail -20 $O/sigchurn.err; exit 1; }
      show $O/sigchurn.json sigchurn value ms_per_step parity_vs_labels stage_ms key_tiers ;;
    churntrace)
      timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --hip-trace --stats -d $O/ct -o run -- python bench.py --clients 16000 --steps 8 --warmup 3 --cpu-threads 0 --no-pcie --no-latency > $O/ct.json 2> $O/ct.err \
        || { echo churntrace failed; tail -20 $O/ct.err; exit 1; }
      echo churntrace ok ;;
    mvccpmc)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/pmc_fetch -o run -- python bench.py --workload mvcc --steps 10 --warmup 2 > $O/pmc_fetch.json 2> $O/pmc_fetch.err \
        && timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run -- python bench.py --workload mvcc --steps 10 --warmup 2 > $O/pmc_write.json 2> $O/pmc_write.err \
        || { echo mvccpmc failed; exit 1; }
      echo mvccpmc ok ;;
    fetchcalib)
      # FETCH_SIZE against known bytes: a streaming read and random 64 B gathers (tools/fetch_calib.py)
      timeout -s KILL 120 rocprofv3 --output-format csv --kernel-trace --pmc FETCH_SIZE -d $O/fcal -o run -- python tools/fetch_calib.py > $O/fcal.out 2>&1 \
        || { echo fetchcalib failed; tail -20 $O/fcal.out; exit 1; }
      python3 tools/fetch_calib_report.py $O/fcal/run_counter_collection.csv | tee $O/fcal_report.txt ;;
    pipeline)
      timeout -k 10 400 python -u bench.py --workload pipeline --steps 12 --warmup 2 > $O/pipeline.json 2> $O/pipeline.err \
        || { echo pipeline failed; tail -20 $O/pipeline.err; exit 1; }
      show $O/pipeline.json pipeline value ms_per_step parity_vs_labels stage_ms_per_step latency_1block_ms ;;
    mvcc)
      timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err \
        || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
      show $O/mvcc.json mvcc value ms_per_step parity_vs_labels stage_ms single_block_calls ;;
    sig)
      timeout -k 10 300 python -u bench.py --workload sig --steps 10 --warmup 2 > $O/sig.json 2> $O/sig.err \
        || { echo sig failed; tail -20 $O/sig.err; exit 1; }
      show $O/sig.json sig value ms_per_step parity_vs_labels ;;
    c5)
      timeout -k 10 400 python -u bench.py --workload c5 --steps 10 --warmup 2 > $O/c5.json 2> $O/c5.err \
        || { echo c5 failed; tail -20 $O/c5.err; exit 1; }
      show $O/c5.json c5 value ms_per_step parity_vs_labels host_ms ;;
    sbe)
      timeout -k 10 400 python -u tools/bench_sbe.py > $O/sbe.json 2> $O/sbe.err || { echo bench_sbe failed; tail -20 $O/sbe.err; exit 1; }
      tail -c 400 $O/sbe.json; echo ;;
    trace)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/st -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/st.json 2> $O/st.err \
        || { echo trace failed; tail -20 $O/st.err; exit 1; }
      echo trace ok ;;
    notorch)
      timeout -k 10 400 python -u tools/bench_notorch.py > $O/notorch.json 2> $O/notorch.err \
        || { echo notorch failed; tail -20 $O/notorch.err; exit 1; }
      show $O/notorch.json notorch value ms_per_step parity_vs_labels torch_loaded ;;
    notorch2)
      timeout -k 10 400 python -u tools/bench_notorch.py --contexts 2 > $O/notorch2.json 2> $O/notorch2.err \
        || { echo notorch2 failed; tail -20 $O/notorch2.err; exit 1; }
      show $O/notorch2.json notorch2 value ms_per_step per_context_ms_per_step parity_vs_labels ;;
    mvcctrace)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --hip-trace --stats -d $O/mt -o run -- python bench.py --workload mvcc --steps 40 --warmup 2 --mvcc-single-steps 0 > $O/mt.json 2> $O/mt.err \
        || { echo mvcctrace failed; tail -20 $O/mt.err; exit 1; }
      echo mvcctrace ok ;;
    pipetrace)
      timeout -k 10 400 rocprofv3 --output-format csv --kernel-trace --hip-trace --stats -d $O/pt -o run -- python bench.py --workload pipeline --steps 6 --warmup 2 --pipeline-latency-blocks 4 > $O/pt.json 2> $O/pt.err \
        || { echo pipetrace failed; tail -20 $O/pt.err; exit 1; }
      echo pipetrace ok ;;
    apitrace)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --hip-trace -d $O/at -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/at.json 2> $O/at.err \
        || { echo apitrace failed; tail -20 $O/at.err; exit 1; }
      echo apitrace ok ;;
    pcietrace)
      # the PCIe-inclusive rotation's copies and kernels (tools/copy_trace.py reads the CSVs)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $O/pcie -o run -- python bench.py --steps ${PCIE_STEPS:-20} --warmup 3 --cpu-threads 0 --no-latency > $O/pcie.json 2> $O/pcie.err \
        || { echo pcietrace failed; tail -20 $O/pcie.err; exit 1; }
      python3 tools/copy_trace.py $O/pcie > $O/pcie_summary.txt 2>&1; tail -25 $O/pcie_summary.txt ;;
    pcietrace2)
      # copies only (no kernel trace): the unprofiled kernels' timing, the copies' timeline
      BENCH_STEPLOG=1 timeout -k 10 300 rocprofv3 --output-format csv --memory-copy-trace -d $O/pcie2 -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency > $O/pcie2.json 2> $O/pcie2.err \
        || { echo pcietrace2 failed; tail -20 $O/pcie2.err; exit 1; }
      grep "steps ms\|slowest" $O/pcie2.err | tail -2
      python3 tools/copy_trace.py $O/pcie2 > $O/pcie2_summary.txt 2>&1; tail -28 $O/pcie2_summary.txt ;;
    rehearse2)
      # two ranks of the shard protocol on the one GPU (gloo between them; the driver runs the real
      # N=2..8 over RCCL): per-rank step and device time against N=1 through the same protocol
      timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie --shard-protocol \
        > $O/n1_shard.json 2> $O/n1_shard.err || { echo rehearse2 n1 failed; tail -20 $O/n1_shard.err; exit 1; }
      FGV_BENCH_SAME_DEVICE=1 FGV_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 \
        --cpu-threads 0 --no-latency --no-pcie > $O/n2_same.json 2> $O/n2_same.err \
        || { echo rehearse2 n2 failed; tail -20 $O/n2_same.err; exit 1; }
      grep "ms per step, device batch" $O/n1_shard.err $O/n2_same.err
      show $O/n2_same.json n2 value ms_per_step parity_vs_labels ;;
    pciesteps*)
      # unprofiled PCIe passes at 12 / 20 / 40 timed steps with per-step host timings (BENCH_STEPLOG);
      # pciesteps<W>: W warmup steps (default 3)
      w=${step#pciesteps}; w=${w:-3}
      for k in 12 20 40; do
        BENCH_STEPLOG=1 timeout -k 10 300 python -u bench.py --steps $k --warmup $w --cpu-threads 0 --no-latency > $O/pcies_$k.json 2> $O/pcies_$k.err \
          || { echo pciesteps failed; tail -20 $O/pcies_$k.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/pcies_$k.json')); p=d['pcie_inclusive']; print('pcie steps $k', d['ms_per_step'], p['ms_per_step'])"
        grep "steps ms\|slowest\|median step" $O/pcies_$k.err | tail -3
      done ;;
    pcie*)
      # pcie<N>: N runs of the default bench's PCIe-inclusive pass (lean: no CPU baseline / latency)
      n=${step#pcie}; n=${n:-1}
      for rep in $(seq 1 $n); do
        timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency > $O/pcie_$rep.json 2> $O/pcie_$rep.err \
          || { echo pcie failed; tail -20 $O/pcie_$rep.err; exit 1; }
        python3 -c "import json; d=json.load(open('$O/pcie_$rep.json')); p=d['pcie_inclusive']; print('pcie $rep', d['ms_per_step'], p['ms_per_step'], p['h2d_GBps'], p['parity_vs_labels'])"
      done ;;
    latapi)
      # the single-block chain with the HIP API trace: when the host enqueued each kernel
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --hip-trace -d $O/latapi -o run -- python tools/latency_probe.py > $O/latapi.out 2> $O/latapi.err \
        || { echo latapi failed; tail -20 $O/latapi.err; exit 1; }
      tail -1 $O/latapi.out ;;
    lattrace)
      timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats -d $O/lat -o run -- python tools/latency_probe.py > $O/lat.out 2> $O/lat.err \
        || { echo lattrace failed; tail -20 $O/lat.err; exit 1; }
      tail -1 $O/lat.out ;;
    profileblock)
      # the block workload's stats + PMC passes only (tools/profile_round.sh's block lines)
      P="rocprofv3 --output-format csv"; D=$O/prof; mkdir -p $D
      timeout -k 10 300 $P --kernel-trace --stats -d $D/block -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $D/block.json 2> $D/block.err \
        && timeout -k 10 300 $P --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $D/pmc_blk_valu -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $D/pmc_blk_valu.json 2> $D/pmc_blk_valu.err \
        && timeout -k 10 300 $P --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $D/pmc_blk_fetch -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $D/pmc_blk_fetch.json 2> $D/pmc_blk_fetch.err \
        && timeout -k 10 300 $P --kernel-trace --pmc WRITE_SIZE -d $D/pmc_blk_write -o run -- python bench.py --steps 5 --warmup 1 --cpu-threads 0 --no-pcie --no-latency > $D/pmc_blk_write.json 2> $D/pmc_blk_write.err \
        || { echo profileblock failed; exit 1; }
      echo profileblock ok ;;
    profile)
      PROF_OUT=$O/prof bash tools/profile_round.sh || { echo profile failed; exit 1; } ;;
    with:*)
      # with:VAR=VAL:<step> -- any other step with VAR=VAL set (its output under <out>/<VAR_VAL>/)
      spec=${step#with:}; kv=${spec%%:*}; sub=${spec#*:}; tag=$(echo $kv | tr '=' '_')
      env $kv bash "$0" "${O#gpurun_out/}/$tag" "$sub" || exit 1 ;;
    py:*)
      f=${step#py:}
      timeout -k 10 300 python -u $f > $O/$(basename $f).out 2>&1 || { echo "$f failed"; tail -30 $O/$(basename $f).out; exit 1; }
      tail -20 $O/$(basename $f).out ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
