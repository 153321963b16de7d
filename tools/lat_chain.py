"""Single-block chain from a rocprofv3 kernel-trace CSV of tools/latency_probe.py (profiling aid,
DESIGN.md s5c): per call, every kernel's start / end relative to the call's first kernel, the
queue it ran on, and the medians over calls -- which launches sit on the critical chain and how
long each waits behind its predecessor.

usage: python tools/lat_chain.py <run_kernel_trace.csv> [first-kernel-name]
"""
import csv
import statistics as S
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else 'k_bd_parse'
rows.sort(key=lambda r: int(r['Start_Timestamp']))
nm = lambda r: r['Kernel_Name'].split('(')[0].split('<')[0]
starts = [i for i, r in enumerate(rows) if nm(r) == first]
calls = []
for a, b in zip(starts, starts[1:] + [len(rows)]):
    calls.append(rows[a:b])
calls = calls[3:]  # warmup
stat = {}
order = []
for c in calls:
    t0 = int(c[0]['Start_Timestamp'])
    seen = {}
    for r in c:
        k = nm(r)
        seen[k] = seen.get(k, 0) + 1
        key = k if seen[k] == 1 else '%s#%d' % (k, seen[k])
        if key not in stat:
            stat[key] = []
            order.append(key)
        stat[key].append(((int(r['Start_Timestamp']) - t0) / 1e3, (int(r['End_Timestamp']) - t0) / 1e3,
                          r.get('Queue_Id', '?')))
ends = [max(int(r['End_Timestamp']) for r in c) - int(c[0]['Start_Timestamp']) for c in calls]
print('calls: %d, first kernel -> last kernel end: median %.1f us' % (len(calls), S.median(ends) / 1e3))
print('%-26s %5s %9s %9s %9s  queue' % ('kernel', 'n', 'start', 'end', 'dur'))
for k in sorted(order, key=lambda k: S.median(s for s, _, _ in stat[k])):
    v = stat[k]
    if len(v) < len(calls) // 2:
        continue
    print('%-26s %5d %9.1f %9.1f %9.1f  %s' % (k, len(v), S.median(s for s, _, _ in v), S.median(e for _, e, _ in v),
                                                S.median(e - s for s, e, _ in v), v[0][2]))
