#!/bin/bash
# round 3: key-level batches on the device fold (tools/bench_sbe.py), the default bench, a clean
# block-step kernel profile (init kernels excluded), and the PCIe pass with blit-kernel copies
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_mvcc.py tests/test_gpu_rangequery.py tests/test_gpu_ledgers.py tests/test_gpu_sbe.py > $O/tests.log 2>&1 || { echo tests failed; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/bench_sbe.py > $O/sbe.json 2> $O/sbe.err || { echo bench_sbe failed; tail -20 $O/sbe.err; exit 1; }
cat $O/sbe.json
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['parity_vs_labels'], d['roofline']['frac'], d['pcie_inclusive']['ms_per_step'], d['cpu_baseline']['value'], d['cpu_baseline']['one_thread'], d['kernel_ms'])"
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --stats --kernel-exclude-regex "k_gtab|k_keytab" -d $O/blockprof -o run -- python bench.py --steps 20 --warmup 3 --cpu-threads 0 --no-latency --no-pcie > $O/blockprof.json 2> $O/blockprof.err || { echo blockprof failed; tail -20 $O/blockprof.err; exit 1; }
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --steps 12 --warmup 2 --cpu-threads 0 --no-latency > $O/nosdma.json 2> $O/nosdma.err || { echo nosdma failed; tail -20 $O/nosdma.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/nosdma.json')); print('nosdma', d['value'], d['ms_per_step'], d['pcie_inclusive'])"
for rep in 1 2; do
  for tv in 1 0; do
    FGV_MVX_TOUCH=$tv timeout -k 10 300 python -u bench.py --workload mvcc > $O/mvcc_t${tv}_$rep.json 2> $O/mvcc_t${tv}_$rep.err || { echo mvcc failed; tail -20 $O/mvcc_t${tv}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/mvcc_t${tv}_$rep.json')); print('mvcc touch $tv rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
    FGV_MVX_ONEWALK=$tv timeout -k 10 300 python -u bench.py --workload mvcc > $O/mvcc_w${tv}_$rep.json 2> $O/mvcc_w${tv}_$rep.err || { echo mvcc failed; tail -20 $O/mvcc_w${tv}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/mvcc_w${tv}_$rep.json')); print('mvcc onewalk $tv rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'])"
    FGV_PARSE_TOUCH=$tv timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --cpu-threads 0 --no-pcie --no-latency > $O/parse_t${tv}_$rep.json 2> $O/parse_t${tv}_$rep.err || { echo parse ab failed; tail -20 $O/parse_t${tv}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/parse_t${tv}_$rep.json')); print('parse touch $tv rep $rep', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['kernel_ms']['k_bd_parse'])"
  done
done
echo done
