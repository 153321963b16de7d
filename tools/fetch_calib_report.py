"""Report of tools/fetch_calib.py under rocprofv3 --pmc FETCH_SIZE: per kernel, the counter (KB)
against the bytes the kernel must read, i.e. the factor that turns FETCH_SIZE into bytes for
that access shape on gfx950.

usage: python tools/fetch_calib_report.py <run_counter_collection.csv>
"""
import csv
import statistics as S
import sys

STREAM = 1 << 30          # table.sum() over 1 GiB
GATHER = (1 << 20) * 64   # 1M random 64 B rows (index_select)
vals = {}
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Counter_Name") != "FETCH_SIZE":
        continue
    k = r["Kernel_Name"]
    vals.setdefault((k, r["Dispatch_Id"]), 0.0)
    vals[(k, r["Dispatch_Id"])] += float(r["Counter_Value"])
per = {}
for (k, _), v in vals.items():
    per.setdefault(k, []).append(v)
for k, v in sorted(per.items(), key=lambda kv: -max(kv[1])):
    kb = S.median(v)
    if kb < 16 * 1024:
        continue
    name = k.split("(")[0][:90]
    for label, want in (("stream 1 GiB", STREAM), ("gather 64 MiB in 64 B rows", GATHER)):
        ratio = want / (kb * 1024)
        if 0.2 < ratio < 5:
            print(f"{name}: FETCH_SIZE {kb / 1024:.1f} MB over {len(v)} dispatches; {label}: bytes / counter = {ratio:.2f}")
