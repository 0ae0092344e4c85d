"""The c3_batch64 entry of profiles/sgns_pmc.json from two rocprofv3 counter passes (FETCH_SIZE,
WRITE_SIZE) over `bench.py --batch-walks 64 --steps S --warmup W ...` (scripts/gpu_r05y.sh).

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE and WRITE_SIZE in KiB; FETCH_SIZE reads half), as
scripts/rocprof_summary.py applies to the headline. Per kernel: the mean over its dispatches,
and launches per step = dispatches / (steps + warmup). bench.py reads the entry's
hbm_bytes_per_launch (= hbm_bytes_per_step: one launch of the graphed step) as the batch64
roofline's `traffic`.

Usage: python scripts/pmc_batch64.py <fetch.csv> <write.csv> <steps+warmup> <round> <note>"""
import collections
import csv
import json
import sys

PMC = 'profiles/sgns_pmc.json'


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r['Counter_Name'] != counter:
            continue
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        if name.startswith('void '):
            name = name[5:]
        name = name.split('(')[0]
        acc[name].append(float(r['Counter_Value']))
    return acc


def main():
    fetch_csv, write_csv, n_steps, rnd, note = sys.argv[1:6]
    n_steps = int(n_steps)
    fe, wr = per_kernel(fetch_csv, 'FETCH_SIZE'), per_kernel(write_csv, 'WRITE_SIZE')
    keep = ('k_out', 'k_place', 'k_touch', 'k_rows_adam', 'k_sgns_g16', 'k_lazy_boundary',
            'k_walk', 'k_step_expand')
    out, total = {}, 0.0
    for k in sorted(set(fe) & set(wr)):
        if not k.startswith(keep):
            continue
        f = 1024.0 * sum(fe[k]) / len(fe[k])
        w = 1024.0 * sum(wr[k]) / len(wr[k])
        per_step = len(fe[k]) / n_steps
        out[k] = {'fetch_bytes': round(f), 'write_bytes': round(w),
                  'hbm_bytes': round(2 * f + w), 'launches_per_step': round(per_step, 3)}
        total += (2 * f + w) * per_step
    d = json.load(open(PMC))
    d['entries'] = [e for e in d['entries'] if e.get('workload') != 'c3_batch64']
    d['entries'].append({'round': rnd, 'workload': 'c3_batch64', 'note': note,
                         'hbm_bytes_per_kernel': out, 'hbm_bytes_per_step': round(total),
                         'hbm_bytes_per_launch': round(total)})
    json.dump(d, open(PMC, 'w'), indent=1)
    print(json.dumps({'hbm_bytes_per_step': round(total),
                      'k_out_rows': {k: v for k, v in out.items() if k.startswith('k_out_rows')}}))


if __name__ == '__main__':
    main()
