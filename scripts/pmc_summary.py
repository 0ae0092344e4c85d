"""Per-kernel HBM bytes (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter_collection.csv) of the
dispatches whose kernel name matches the step's kernels: mean per dispatch, in MB (the counters
report KB). Usage: python scripts/pmc_summary.py fetch.csv write.csv"""
import collections
import csv
import re
import sys


def per_kernel(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(path)):
        d = int(r['Dispatch_Id'])
        per[d][r['Counter_Name']] += float(r['Counter_Value'])
        kn = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        name[d] = re.sub(r'\(.*', '', kn).replace('void ', '')
    out = collections.defaultdict(list)
    for d, c in per.items():
        for v in c.values():
            out[name[d]].append(v / 1024.0)   # KB -> MB
    return out


fetch, write = per_kernel(sys.argv[1]), per_kernel(sys.argv[2])
rows = []
for k in sorted(set(fetch) | set(write)):
    f, w = fetch.get(k, []), write.get(k, [])
    if not f and not w:
        continue
    fm = sum(f) / len(f) if f else 0.0
    wm = sum(w) / len(w) if w else 0.0
    rows.append((fm + wm, k, len(f), fm, wm))
print(f"{'kernel':70s} {'n':>5s} {'FETCH MB':>10s} {'WRITE MB':>10s}")
for _, k, n, fm, wm in sorted(rows, reverse=True)[:24]:
    print(f"{k[:70]:70s} {n:5d} {fm:10.2f} {wm:10.2f}")
