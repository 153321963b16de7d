"""PCIe-inclusive rotation from a rocprofv3 --memory-copy-trace --kernel-trace run of bench.py
(profiling aid): the batch-sized host-to-device copies in time order -- duration,
GB/s, the idle link between consecutive copies -- and what the GPU ran during each idle gap.

usage: python tools/copy_trace.py <rocprofv3 output dir>
"""
import csv
import glob
import os
import statistics as S
import sys

d = sys.argv[1]
mc = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if not mc:
    sys.exit("no memory_copy_trace.csv under %s" % d)
rows = list(csv.DictReader(open(mc[0])))
kern = list(csv.DictReader(open(kt[0]))) if kt else []
kern.sort(key=lambda r: int(r["Start_Timestamp"]))


def size(r):
    for k in ("Bytes", "Size", "Copy_Bytes"):
        if k in r and r[k]:
            return int(r[k])
    return 0


h2d = [r for r in rows if "HOST_TO_DEVICE" in (r.get("Direction", "") + r.get("Kind", "") + r.get("Operation", "")).upper()]
big = [r for r in h2d if size(r) >= 16 << 20]
big.sort(key=lambda r: int(r["Start_Timestamp"]))
print("columns:", list(rows[0].keys()) if rows else None)
print("H2D copies: %d, batch-sized (>= 16 MiB): %d" % (len(h2d), len(big)))
gaps, durs, rates = [], [], []
prev = None
for r in big:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    durs.append((e - s) / 1e3)
    rates.append(size(r) / max(e - s, 1))  # bytes/ns = GB/s
    if prev is not None:
        gaps.append(((s - prev) / 1e3, prev, s))
    prev = e
if durs:
    print("copy duration us: med %.1f min %.1f max %.1f; GB/s med %.1f" % (S.median(durs), min(durs), max(durs), S.median(rates)))
if gaps:
    g = [x[0] for x in gaps]
    print("idle link between batch copies us: med %.1f p90 %.1f max %.1f (n=%d)" % (S.median(g), sorted(g)[len(g) * 9 // 10], max(g), len(g)))
    span = (int(big[-1]["End_Timestamp"]) - int(big[0]["Start_Timestamp"])) / 1e3
    print("link busy over the pass: %.1f %% of %.1f us" % (100 * sum(durs[1:]) / span if span else 0, span))
    print("--- the largest gaps: kernels that started inside them")
    for gap, a, b in sorted(gaps, reverse=True)[:5]:
        ks = [x["Kernel_Name"].split("(")[0] for x in kern if a <= int(x["Start_Timestamp"]) < b]
        print("%8.1f us: %s" % (gap, ", ".join(ks[:12])))
