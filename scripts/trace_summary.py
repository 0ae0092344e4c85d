"""Kernel-trace summary (rocprofv3 --kernel-trace CSV): per-kernel dispatch counts and mean
duration, and with `timeline` the kernel sequence of one step. Usage:
    python scripts/trace_summary.py <kernel_trace.csv> [timeline]"""
import csv, collections, re, sys
rows=list(csv.DictReader(open(sys.argv[1])))
def short(n):
    n=n.replace('(anonymous namespace)::','').replace('void ','')
    m=re.match(r'([A-Za-z_:0-9]+)(<[^()]*>)?', n)
    s=m.group(1) if m else n
    if m and m.group(2) and s.startswith('k_'): s+=m.group(2)[:40]
    return s
rows.sort(key=lambda r:int(r['Start_Timestamp']))
stats=collections.defaultdict(list)
for r in rows[len(rows)//2:]:
    stats[short(r['Kernel_Name'])].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(stats.items(), key=lambda kv:-sum(kv[1])):
    print(f"{k[:80]:80s} n={len(v):4d} mean={sum(v)/len(v):8.1f}us tot={sum(v):9.1f}")
if len(sys.argv)>2:
    # timeline of one step in the middle (relative us)
    mid=[r for r in rows if short(r['Kernel_Name']).startswith('k_sgns_g16')]
    a=int(mid[len(mid)//2]['Start_Timestamp'])
    seq=[r for r in rows if a-300000 < int(r['Start_Timestamp']) < a+300000]
    for r in seq:
        print(f"{(int(r['Start_Timestamp'])-a)/1e3:9.1f} {(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:7.1f} q{r['Queue_Id']} {short(r['Kernel_Name'])[:70]}")
