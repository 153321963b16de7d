"""Per-step critical-chain statistics from a rocprofv3 kernel-trace CSV of a C2 bench run
(profiling aid): the main-queue kernels after each k_point28 (wait before each,
duration), then the next batch's front half relative to k_bd_emit.

usage: python tools/trace_chain.py <run_kernel_trace.csv>
"""
import csv
import statistics as S
import sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
q1 = [r for r in rows if r.get('Queue_Id') == rows[[i for i,r in enumerate(rows) if r['Kernel_Name'].startswith('k_point28')][0]]['Queue_Id']]
names = [r['Kernel_Name'].split('(')[0] for r in q1]
res = {}
for i, r in enumerate(q1):
    if names[i] != 'k_point28': continue
    seq = q1[i:i+12]
    t0 = int(r['Start_Timestamp'])
    prev_end = None
    for k, x in enumerate(seq):
        nm = x['Kernel_Name'].split('(')[0]
        st, en = int(x['Start_Timestamp']) - t0, int(x['End_Timestamp']) - t0
        key = f"{k:02d} {nm}"
        res.setdefault(key, []).append((st - (prev_end if prev_end is not None else st), en - st))
        prev_end = en
for k in sorted(res):
    v = res[k]
    if len(v) < 5: continue
    print("%-32s n=%3d  wait-before med %6.1f  dur med %6.1f  dur p90 %6.1f" % (k, len(v), S.median(a for a, _ in v)/1e3, S.median(b for _, b in v)/1e3, sorted(b for _, b in v)[int(len(v)*0.9)]/1e3))

print('--- front half of the next batch, per step (us)')
rows = list(csv.DictReader(open(sys.argv[1]))); rows.sort(key=lambda r:int(r['Start_Timestamp']))
def ts(r): return int(r['Start_Timestamp'])/1e3
def te(r): return int(r['End_Timestamp'])/1e3
nm=lambda r:r['Kernel_Name'].split('(')[0]
em=[r for r in rows if nm(r)=='k_bd_emit']
pa=[r for r in rows if nm(r)=='k_bd_parse']
pay=[r for r in rows if nm(r)=='k_bd_sha_payload']
co=[r for r in rows if nm(r)=='k_bd_count']
idn=[r for r in rows if nm(r)=='k_bd_ident']
pt=[r for r in rows if nm(r)=='k_point28']
out={k:[] for k in ['emit->parse','parse dur','parse->ident','ident dur','count end->emit','step','pay dur','emit->pay']}
for i in range(len(em)-1):
    e0=ts(em[i]); e1=ts(em[i+1])
    p=[r for r in pa if e0<ts(r)<e1]; c=[r for r in co if e0<ts(r)<e1]; d=[r for r in idn if e0<ts(r)<e1]; y=[r for r in pay if e0<ts(r)<e1]
    if not(p and c and d and y): continue
    p,c,d,y=p[0],c[0],d[0],y[0]
    out['emit->parse'].append(ts(p)-e0); out['parse dur'].append(te(p)-ts(p)); out['parse->ident'].append(ts(d)-te(p))
    out['ident dur'].append(te(d)-ts(d)); out['count end->emit'].append(e1-te(c)); out['step'].append(e1-e0)
    out['pay dur'].append(te(y)-ts(y)); out['emit->pay'].append(ts(y)-e0)
for k,v in out.items(): print("%-16s n=%3d med %7.1f p10 %7.1f p90 %7.1f"%(k,len(v),S.median(v),sorted(v)[len(v)//10],sorted(v)[len(v)*9//10]))
