"""Summarise rocprofv3 output (gpurun_out/prof_*) into profiles/ (committed evidence).

    python scripts/rocprof_summary.py <round-tag> [pairs_per_launch]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, verbatim), profiles/<tag>_pmc.json
(per-kernel mean FETCH_SIZE / WRITE_SIZE / TCC_EA0_ATOMIC_sum per dispatch) and
profiles/sgns_pmc.json (what bench.py reads for roofline.traffic).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB;
FETCH_SIZE reads 1/2 of a wide coalesced stream's bytes on gfx950 (doubled here — calibrated
on k_adam, whose 4 x 1 GiB read stream reports 2 GiB), WRITE_SIZE is exact for float atomics
and 16-B streaming stores; TCC_EA0_ATOMIC_sum counts 64-B atomic requests.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, 'gpurun_out')
PROF = os.path.join(REPO, 'profiles')
KERNELS = {'k_sgns': 'dw_sgns_walks', 'k_adam': 'dw_adam_dense',
           'k_walk_deepwalk_fast': 'dw_walk_fast/deepwalk',
           'k_walk_node2vec_fast': 'dw_walk_fast/node2vec', 'k_sgns_rec': 'dw_sgns_records',
           'k_out_adam': 'dw_adam_out_gather'}


def short(name):
    for k in sorted(KERNELS, key=len, reverse=True):
        if k + '<' in name or k + '(' in name:
            return k
    return None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r01'
    pairs = int(sys.argv[2]) if len(sys.argv) > 2 else None
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, 'prof_trace', '**', '*kernel_stats.csv'), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, f'{tag}_kernel_stats.csv'))
    avg_ns = {}
    if stats:
        for r in csv.DictReader(open(stats[0])):
            k = short(r['Name'])
            if k:
                avg_ns[k] = float(r['AverageNs'])
    pmc = collections.defaultdict(dict)
    for path in glob.glob(os.path.join(OUT, 'prof_pmc_*', '**', '*counter_collection.csv'),
                          recursive=True):
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            k = short(r['Kernel_Name'])
            if k:
                vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
        for k, d in vals.items():
            for ctr, v in d.items():
                pmc[k][ctr] = sum(v) / len(v)
    summary = {}
    for k, d in pmc.items():
        e = dict(d)
        fetch, write = d.get('FETCH_SIZE'), d.get('WRITE_SIZE')
        if fetch is not None and write is not None:
            e['hbm_bytes_per_launch'] = 2 * fetch * 1024 + write * 1024
        if 'TCC_EA0_ATOMIC_sum' in d:
            e['atomic_bytes_per_launch'] = d['TCC_EA0_ATOMIC_sum'] * 64
        if k in avg_ns:
            e['avg_ns'] = avg_ns[k]
            if 'hbm_bytes_per_launch' in e:
                e['hbm_GBps'] = e['hbm_bytes_per_launch'] / avg_ns[k]
            if 'atomic_bytes_per_launch' in e:
                e['atomic_GBps'] = e['atomic_bytes_per_launch'] / avg_ns[k]
        summary[KERNELS.get(k, k)] = e
    with open(os.path.join(PROF, f'{tag}_pmc.json'), 'w') as f:
        json.dump(summary, f, indent=2)
    s = summary.get('dw_sgns_walks')
    if s and 'hbm_bytes_per_launch' in s and pairs:
        with open(os.path.join(PROF, 'sgns_pmc.json'), 'w') as f:
            json.dump({'round': tag, 'pairs_per_launch': pairs,
                       'hbm_bytes_per_launch': s['hbm_bytes_per_launch'],
                       'atomic_bytes_per_launch': s.get('atomic_bytes_per_launch'),
                       'note': '2*FETCH_SIZE + WRITE_SIZE (KiB->B); see scripts/rocprof_summary.py'},
                      f, indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == '__main__':
    main()
