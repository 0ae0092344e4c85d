"""The exact node2vec walker's per-edge position index at C5 (R-MAT 24, 256M edge draws):
its size under several encodings, its build time and the walker's rate.

    python scripts/microbench/n2v_index_c5.py [--scale 24] [--edges 256000000] [--walks 1048576]

Prints one JSON line per stage (graph, counts, sizes, build, rates) so a long run shows progress.
"""
import argparse
import json
import os
import random
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'deepwalk-and-node2vec_amd'))

from shallow_encoders.graph.random_walk_generator import Node2Vec  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402
from shallow_encoders.graph.rng import draw_uniforms  # noqa: E402


def emit(**kw):
    print(json.dumps(kw), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scale', type=int, default=24)
    ap.add_argument('--edges', type=int, default=256_000_000)
    ap.add_argument('--walks', type=int, default=1_048_576)
    ap.add_argument('--check-walks', type=int, default=4096)
    ap.add_argument('--L', type=int, default=80)
    ap.add_argument('--p', type=float, default=0.25)
    ap.add_argument('--q', type=float, default=4.0)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    t0 = time.perf_counter()
    csr = rmat_graph(args.scale, args.edges, 0, device=dev)
    torch.cuda.synchronize(dev)
    V, E = csr.vocab_size, csr.nnz
    emit(stage='graph', V=V, directed_edges=E, seconds=time.perf_counter() - t0)
    csr.device_tensors(dev, need_sorted=True, need_adj_pos=True, need_hub_bits=True)
    torch.cuda.synchronize(dev)
    a = time.perf_counter()
    d = csr.device_tensors(dev, need_edge_cn=True)
    torch.cuda.synchronize(dev)
    emit(stage='counts', edge_cn_build_ms=(time.perf_counter() - a) * 1e3,
         hubs_with_bitmaps=int((d['hub_idx'] >= 0).sum()))

    cn = d['edge_cn'][:E].to(torch.int64) & 0x7FFFFFFF    # bit 31: t in N(v); bits 0-30: C
    deg = d['row_ptr'][1:] - d['row_ptr'][:-1]
    deg_t = deg[d['col'][:E].long()]                  # deg(v) of every directed edge t -> v
    n_pos = int(cn.sum())
    q = torch.tensor([0.5, 0.9, 0.99, 0.999, 0.9999], dtype=torch.float64, device=dev)
    samp = cn[torch.randint(0, E, (1 << 23,), device=dev)].double()
    u16 = deg_t <= 65536
    by_u16 = int((torch.where(u16, 2, 4) * cn).sum())
    bitmap = (deg_t + 7) // 8                         # a deg(v)-bit mask of the common positions
    hyb = int(torch.minimum(4 * cn, bitmap + bitmap // 8 + 4).sum())
    hyb16 = int(torch.minimum(torch.where(u16, 2, 4) * cn, bitmap + bitmap // 8 + 4).sum())
    emit(stage='sizes', entries=n_pos, fits_u32_offsets=n_pos < (1 << 32),
         edges_with_common=int((cn > 0).sum()), max_common=int(cn.max()),
         max_degree=int(deg.max()), quantiles_common=dict(zip(
             ['p50', 'p90', 'p99', 'p999', 'p9999'],
             [float(x) for x in torch.quantile(samp, q)])),
         bytes_int32=4 * n_pos + 32 * E, bytes_u16_where_deg_le_65536=by_u16 + 32 * E,
         bytes_hybrid_bitmap=hyb + 32 * E, bytes_hybrid_bitmap_u16=hyb16 + 32 * E,
         records_bytes=32 * E, free_hbm=torch.cuda.mem_get_info(dev)[0])
    del cn, deg, deg_t, samp, u16, bitmap
    torch.cuda.empty_cache()

    os.environ.setdefault('DW_N2V_INDEX_BYTES', str(200 << 30))
    a = time.perf_counter()
    d = csr.device_tensors(dev, need_n2v_index=True)
    torch.cuda.synchronize(dev)
    info = dict(d.get('n2v_index_info', {}))
    emit(stage='build', seconds=time.perf_counter() - a, **info)
    if d.get('n2v_rec') is None:   # the wave walker with the per-edge counts (the fallback)
        L, n = args.L, args.check_walks
        w = Node2Vec(csr, L, p=args.p, q=args.q, device=dev)
        st = (torch.randperm(V - 1, generator=torch.Generator().manual_seed(1))[:n] + 1).to(
            torch.int32).to(dev)
        u = torch.from_numpy(draw_uniforms(n * (L - 1), random.Random(0))).to(dev)
        out = torch.empty((n, L), dtype=torch.int32, device=dev)
        w.walk_batch(st[:64], uniforms=u[:64 * (L - 1)], out=out[:64])
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        w.walk_batch(st, uniforms=u, out=out, check=False)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        c = w.count_replay_traffic(st, u, out=torch.empty_like(out))
        emit(stage='rate', walker='dw_walk_replay_indexed (wave walker, per-edge counts)',
             walks=n, kernel_ms=ms, walks_per_s=n / (ms * 1e-3),
             bytes_per_step=c['bytes'] / max(c['steps'], 1),
             list_entries_per_step=c['entries'] / max(c['steps'], 1),
             hash_probes_per_step=c['probes'] / max(c['steps'], 1))
        return

    L = args.L
    w = Node2Vec(csr, L, p=args.p, q=args.q, device=dev)
    gen = random.Random(0)
    n = args.walks
    st = (torch.randperm(V - 1, generator=torch.Generator().manual_seed(1))[:n] + 1).to(
        torch.int32).to(dev)
    u = torch.from_numpy(draw_uniforms(n * (L - 1), gen)).to(dev)
    out = torch.empty((n, L), dtype=torch.int32, device=dev)
    w.walk_batch(st[:64], uniforms=u[:64 * (L - 1)], out=out[:64])
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        w.walk_batch(st, uniforms=u, out=out, check=False)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    c = w.count_replay_traffic(st, u, out=torch.empty_like(out))
    emit(stage='rate', walker='dw_walk_replay_positions', walks=n, kernel_ms=best,
         walks_per_s=n / (best * 1e-3), bytes_per_step=c['bytes'] / max(c['steps'], 1),
         entries_per_step=c['entries'] / max(c['steps'], 1), serial_picks=c['probes'],
         frac_hbm=c['bytes'] / (best * 1e-3) / 8e12)
    # the Philox walker over the same index (dw_walk_fast_positions), walks from every start
    wp = Node2Vec(csr, L, p=args.p, q=args.q, rng='philox', seed=3, device=dev)
    wp.walk_batch(st[:64], walk_id0=0, out=out[:64])
    best = None
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        wp.walk_batch(st, walk_id0=0, out=out, check=False)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    c = wp.count_traffic(st, walk_id0=0, out=torch.empty_like(out))
    emit(stage='rate_philox', walker=c.get('walker'), walks=n, kernel_ms=best,
         walks_per_s=n / (best * 1e-3), bytes_per_step=c['bytes'] / max(c['steps'], 1),
         position_units_per_step=c.get('position_loads', 0) / max(c['steps'], 1),
         frac_hbm=c['bytes'] / (best * 1e-3) / 8e12)
    w.walk_batch(st, uniforms=u, out=out, check=False)
    # the same walks through the wave walker (DW_N2V_POS=0) on a sample: bit-equal
    k = args.check_walks
    os.environ['DW_N2V_POS'] = '0'
    ref = torch.empty((k, L), dtype=torch.int32, device=dev)
    a = time.perf_counter()
    w.walk_batch(st[:k], uniforms=u[:k * (L - 1)], out=ref)
    torch.cuda.synchronize(dev)
    wave_s = time.perf_counter() - a
    os.environ['DW_N2V_POS'] = '1'
    emit(stage='check', walks=k, equal=bool(torch.equal(ref, out[:k])),
         wave_walker_walks_per_s=k / wave_s)


if __name__ == '__main__':
    main()
