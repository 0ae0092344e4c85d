"""Summarise rocprofv3 output (gpurun_out/prof_*) into profiles/ (committed evidence).

    python scripts/rocprof_summary.py <round-tag> [pairs_per_launch [dim vocab_size [overlap_in
                                      [owner_world in_exchange]]]]

owner_world > 0: a profile of `bench.py --emulate-world W` (rank 0's share of an owner-computes
job of W ranks; the kernels of a real rank, without its collectives); the sgns_pmc.json entry is
then keyed by (owner_world, in_exchange) too, and bench.py reports it as the N = W line's
traffic.

Writes
  profiles/<tag>_kernel_stats.csv  rocprofv3 --stats, verbatim;
  profiles/<tag>_pmc.json          per kernel class: dispatches, mean duration, HBM bytes per
                                   dispatch and per SGNS call (FETCH_SIZE / WRITE_SIZE /
                                   TCC_EA0_ATOMIC_sum passes);
  profiles/sgns_pmc.json           what bench.py reads for roofline.traffic: HBM bytes of one
                                   SGNS step op (pass 1 + sort + pass 2), one entry per
                                   workload (pairs, d, V, scatter, fused out-table Adam,
                                   overlap_in: the in-table k_adam runs inside the op on a
                                   side stream and its bytes count, one dispatch per step).

Kernel classes: one dw_sgns_walks call = one pass-1 dispatch (k_sgns_g16 / k_sgns) + the hipcub
radix-sort dispatches + one k_rec_gather dispatch, so per-call figures divide a class's total
by the number of pass-1 dispatches.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE
reports 1/2 of a wide coalesced stream's bytes on gfx950 (doubled here — calibrated on k_adam,
whose 4 x 1 GiB read stream reports 2 GiB), WRITE_SIZE is exact for float atomics and 16-B
streaming stores; TCC_EA0_ATOMIC_sum counts 64-B atomic requests.
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
SGNS_CLASSES = ('sgns_pass1', 'sgns_sort', 'sgns_pass2')


def kernel_class(name: str):
    if 'k_sgns_g16' in name or 'k_sgns<' in name or 'k_sgns(' in name:
        return 'sgns_pass1'
    if 'k_rec_gather' in name or 'k_adam_rest' in name:   # pass 2 (+ the fused out-table Adam)
        return 'sgns_pass2'
    if 'radix_sort' in name or 'onesweep' in name:
        # the SGNS records sort: u32 row keys, u64 {coef, centre} values; the CSR copy sort
        # (dw_csr_sort_copy, u64 keys only) runs once at setup
        # (the owner form's occurrence sort of the centres, u32/u32 with rocprim's default
        # config, cannot be told from the graph-ingestion sorts by name; it is left out: < 1%
        # of an owner step's bytes)
        return 'sgns_sort' if 'unsigned int, unsigned long' in name else 'csr_sort'
    if any(k in name for k in ('k_occ_keys', 'k_wave_scan', 'k_rec_compact', 'k_rows_adam',
                                'k_rows_gather')):
        # owner-form helpers: centre order, record compaction; lazy in-table exchange: the
        # touched rows' catch-up / gradient gather / update
        return 'sgns_aux'
    for k in ('k_adam', 'k_scale', 'k_walk_deepwalk_fast', 'k_walk_deepwalk_inline',
              'k_walk_node2vec_fast',
              'k_walk_replay', 'k_logits'):
        if k in name:
            return k
    return None


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else 'r01'
    pairs = int(sys.argv[2]) if len(sys.argv) > 2 else None
    dim = int(sys.argv[3]) if len(sys.argv) > 3 else 128          # C3 defaults
    vocab = int(sys.argv[4]) if len(sys.argv) > 4 else 1048577
    overlap_in = bool(int(sys.argv[5])) if len(sys.argv) > 5 else True
    owner_world = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    in_exchange = sys.argv[7] if len(sys.argv) > 7 else None
    os.makedirs(PROF, exist_ok=True)
    stats = glob.glob(os.path.join(OUT, 'prof_trace', '**', '*kernel_stats.csv'), recursive=True)
    dur = collections.defaultdict(lambda: [0, 0.0])   # class -> [calls, total ns]
    if stats:
        shutil.copy(stats[0], os.path.join(PROF, f'{tag}_kernel_stats.csv'))
        for r in csv.DictReader(open(stats[0])):
            k = kernel_class(r['Name'])
            if k:
                dur[k][0] += int(r['Calls'])
                dur[k][1] += float(r['TotalDurationNs'])
    # counter passes: one file per counter group; totals per class and dispatch counts
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for path in glob.glob(os.path.join(OUT, 'prof_pmc_*', '**', '*counter_collection.csv'),
                          recursive=True):
        for r in csv.DictReader(open(path)):
            k = kernel_class(r['Kernel_Name'])
            if not k:
                continue
            ctr = r['Counter_Name']
            tot[k][ctr] += float(r['Counter_Value'])
            disp[k][ctr].add((path, r.get('Dispatch_Id', r.get('Correlation_Id', ''))))
    fused = any('k_adam_rest' in r['Name'] for r in csv.DictReader(open(stats[0]))) \
        if stats else False
    summary = {}
    n_calls_pmc = {}
    for k in set(tot) | set(dur):
        e = {}
        if k in dur:
            e['trace_dispatches'] = dur[k][0]
            e['avg_ns_per_dispatch'] = dur[k][1] / max(dur[k][0], 1)
        per_disp = {}
        for ctr, v in tot[k].items():
            n = len(disp[k][ctr])
            per_disp[ctr] = v / max(n, 1)
            n_calls_pmc[(k, ctr)] = n
        e['counters_per_dispatch'] = per_disp
        if 'FETCH_SIZE' in per_disp and 'WRITE_SIZE' in per_disp:
            e['hbm_bytes_per_dispatch'] = (2 * per_disp['FETCH_SIZE'] +
                                           per_disp['WRITE_SIZE']) * 1024
        if 'TCC_EA0_ATOMIC_sum' in per_disp:
            e['atomic_bytes_per_dispatch'] = per_disp['TCC_EA0_ATOMIC_sum'] * 64
        summary[k] = e
    # per SGNS call: class totals / pass-1 dispatches
    p1 = summary.get('sgns_pass1', {})
    calls_trace = p1.get('trace_dispatches', 0)
    call = {'ms': 0.0, 'hbm_bytes': 0.0}
    ok = calls_trace > 0
    op_classes = SGNS_CLASSES + (('k_adam',) if overlap_in else ()) + \
        (('sgns_aux',) if owner_world else ())
    for k in op_classes:
        e = summary.get(k)
        if not e:
            continue
        if k in dur and calls_trace:
            e['ms_per_sgns_call'] = dur[k][1] / calls_trace / 1e6
            call['ms'] += e['ms_per_sgns_call']
        if 'hbm_bytes_per_dispatch' in e:
            ratio = (n_calls_pmc.get((k, 'FETCH_SIZE'), 0) /
                     max(n_calls_pmc.get(('sgns_pass1', 'FETCH_SIZE'), 0), 1))
            e['hbm_bytes_per_sgns_call'] = e['hbm_bytes_per_dispatch'] * ratio
            call['hbm_bytes'] += e['hbm_bytes_per_sgns_call']
        else:
            ok = False
    summary['dw_sgns_walks_call'] = call
    with open(os.path.join(PROF, f'{tag}_pmc.json'), 'w') as f:
        json.dump(summary, f, indent=2)
    if ok and pairs:
        per_kernel = {k: summary[k].get('hbm_bytes_per_sgns_call') for k in op_classes
                      if k in summary}
        entry = {'round': tag, 'pairs_per_launch': pairs, 'dim': dim, 'vocab_size': vocab,
                 'scatter': 'sorted' if 'sgns_sort' in summary else 'atomic',
                 'fused_out_adam': fused, 'overlap_in': overlap_in,
                 'owner_world': owner_world, 'in_exchange': in_exchange,
                 'hbm_bytes_per_launch': call['hbm_bytes'],
                 'hbm_bytes_per_kernel': per_kernel,
                 'note': '2*FETCH_SIZE + WRITE_SIZE (KiB->B) summed over the kernels of one '
                         'SGNS step op; see scripts/rocprof_summary.py'}
        path = os.path.join(PROF, 'sgns_pmc.json')
        entries = []
        if os.path.exists(path):
            old = json.load(open(path))
            entries = old.get('entries', [old] if 'pairs_per_launch' in old else [])
        key = ('pairs_per_launch', 'dim', 'vocab_size', 'scatter', 'fused_out_adam', 'overlap_in',
               'owner_world', 'in_exchange')
        entries = [e for e in entries if tuple(e.get(k) for k in key) !=
                   tuple(entry[k] for k in key)] + [entry]
        with open(path, 'w') as f:
            json.dump({'entries': entries}, f, indent=2)
    print(json.dumps(summary, indent=2))


if __name__ == '__main__':
    main()
