"""PCIe-inclusive rotation from a rocprofv3 --memory-copy-trace --kernel-trace run of bench.py
(profiling aid).  The trace holds no byte counts, so batch copies are the
host-to-device copies longer than 300 us; bench.py's raw-rate probe (5+1 torch copies, stream 0)
separates the untimed parity pass from the timed pass.  Printed: each timed batch copy (start, end,
idle link before it), the per-step completion times (k_fin_dups ends) and the largest idle gaps with
the kernels that started inside them.

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
T = lambda r, k: int(r[k])  # noqa: E731
t0 = min(T(r, "Start_Timestamp") for r in rows)
big = [r for r in rows if T(r, "End_Timestamp") - T(r, "Start_Timestamp") > 300_000]
probe = [r for r in big if r["Stream_Id"] == "0"]
cut = max(T(r, "End_Timestamp") for r in probe) if probe else t0
timed = sorted((r for r in big if r["Stream_Id"] != "0" and T(r, "Start_Timestamp") >= cut),
               key=lambda r: T(r, "Start_Timestamp"))
print("batch copies in the timed pass: %d" % len(timed))
prev, gaps, durs = None, [], []
for r in timed:
    s, e = T(r, "Start_Timestamp"), T(r, "End_Timestamp")
    g = (s - prev) / 1e3 if prev is not None else 0.0
    durs.append((e - s) / 1e3)
    if prev is not None:
        gaps.append((g, prev, s))
    print("copy %9.3f - %9.3f ms  idle before %7.1f us" % ((s - t0) / 1e6, (e - t0) / 1e6, g))
    prev = e
fd = sorted(T(k, "End_Timestamp") for k in kern if k["Kernel_Name"].startswith("k_fin_dups") and T(k, "End_Timestamp") > cut)
if len(fd) > 1:
    steps = [(b - a) / 1e3 for a, b in zip(fd, fd[1:])]
    print("steps (k_fin_dups to k_fin_dups) us: med %.1f min %.1f max %.1f, n=%d" % (S.median(steps), min(steps), max(steps), len(steps)))
    print("  per step:", " ".join("%.0f" % x for x in steps))
if durs:
    print("batch copy us: med %.1f; idle link med %.1f max %.1f" % (S.median(durs), S.median(g for g, _, _ in gaps) if gaps else 0,
                                                                 max((g for g, _, _ in gaps), default=0)))
for g, a, b in sorted(gaps, reverse=True)[:4]:
    ks = [x["Kernel_Name"].split("(")[0] for x in kern if a <= T(x, "Start_Timestamp") < b]
    print("idle %8.1f us at %.3f ms: %s" % (g, (a - t0) / 1e6, ", ".join(ks[:10])))
