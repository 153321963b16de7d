#!/bin/bash
# round 3: kernel + memory-copy trace of the PCIe-inclusive (host-pinned) C2 pass, and the
# default bench with the chained MVCC defaults
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 300 rocprofv3 --output-format csv --kernel-trace --memory-copy-trace -d $O/tp -o run -- python bench.py --steps 6 --warmup 2 --cpu-threads 0 --no-latency > $O/tp.json 2> $O/tp.err || { echo trace failed; tail -20 $O/tp.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/tp.json')); print(d['value'], d['ms_per_step'], d['pcie_inclusive'])"
timeout -k 10 300 python -u bench.py --workload mvcc --steps 100 --warmup 5 > $O/mvcc.json 2> $O/mvcc.err || { echo mvcc failed; tail -20 $O/mvcc.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/mvcc.json')); print('mvcc', d['value'], d['ms_per_step'], d['parity_vs_labels'], d['stage_ms'], d['single_block_calls'])"
echo done
