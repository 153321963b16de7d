"""Print the kernel + memcpy timeline of the last block step from a rocprofv3 csv trace.
usage: python tools/timeline.py <dir with *_kernel_trace.csv, *_memory_copy_trace.csv> [anchor]"""
import csv
import glob
import sys

d = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_point"
K = list(csv.DictReader(open(glob.glob(d + "/*kernel_trace.csv")[0])))
mfiles = glob.glob(d + "/*memory_copy_trace.csv")
M = list(csv.DictReader(open(mfiles[0]))) if mfiles else []
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K:" + k["Kernel_Name"].split("(")[0]) for k in K]
ev += [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "M:" + m["Direction"]) for m in M]
ev.sort()
idx = [i for i, e in enumerate(ev) if anchor in e[2]]
lo, hi = idx[-2], idx[-1]
t0 = ev[lo][1]
for e in ev[lo:hi + 3]:
    print(f"{(e[0] - t0) / 1e3:9.1f} {(e[1] - t0) / 1e3:9.1f} {(e[1] - e[0]) / 1e3:8.1f}  {e[2]}")
