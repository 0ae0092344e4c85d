"""Kernel rate of the bit-exact replay walkers (rng='python') at C3: uniforms resident in HBM,
HIP events around the launch. DW_LIB_PATH selects an experimental build.

    python scripts/microbench/replay_rates.py [--n2v-walks 65536] [--dw-walks 1048576]
"""
import argparse
import json
import os
import random
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'deepwalk-and-node2vec_amd'))

from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402
from shallow_encoders.graph.rng import draw_uniforms  # noqa: E402


def rate(w, n, L, dev, reps=3):
    gen = random.Random(0)
    st = torch.arange(1, n + 1, dtype=torch.int32, device=dev)
    u = torch.from_numpy(draw_uniforms(n * (L - 1), gen)).to(dev)
    out = torch.empty((n, L), dtype=torch.int32, device=dev)
    w.walk_batch(st[:64], uniforms=u[:64 * (L - 1)], out=out[:64])
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        w.walk_batch(st, uniforms=u, out=out, check=False)
        e1.record()
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return {'walks': n, 'kernel_ms': best, 'walks_per_s': n / (best * 1e-3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n2v-walks', type=int, default=65_536)
    ap.add_argument('--dw-walks', type=int, default=1_048_576)
    ap.add_argument('--L', type=int, default=80)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    csr = rmat_graph(20, 10_000_000, 0, device=dev)
    csr.device_tensors(dev, need_adj_pos=True, need_hub_bits=True, need_sorted=True)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    csr.device_tensors(dev, need_edge_cn=True)   # the per-edge class counts, built once
    e1.record()
    torch.cuda.synchronize(dev)
    res = {'lib': os.environ.get('DW_LIB_PATH', 'default'), 'edge_cn_build_ms': e0.elapsed_time(e1)}
    os.environ['DW_N2V_EDGE_CN'] = '0'
    res['node2vec_p0.25_q4_nocn'] = rate(Node2Vec(csr, args.L, p=0.25, q=4.0, device=dev),
                                         args.n2v_walks, args.L, dev)
    os.environ['DW_N2V_EDGE_CN'] = '1'
    res.update({
           'node2vec_p0.25_q4': rate(Node2Vec(csr, args.L, p=0.25, q=4.0, device=dev),
                                     args.n2v_walks, args.L, dev),
           'node2vec_p0.25_q4_csr': rate(Node2Vec(csr, args.L, p=0.25, q=4.0, device=dev,
                                                  layout='csr'), args.n2v_walks, args.L, dev),
           'node2vec_p1_q1': rate(Node2Vec(csr, args.L, p=1.0, q=1.0, device=dev),
                                  args.n2v_walks, args.L, dev)})
    w = Node2Vec(csr, args.L, p=0.25, q=4.0, device=dev)
    gen = random.Random(0)
    st = torch.arange(1, args.n2v_walks + 1, dtype=torch.int32, device=dev)
    u = torch.from_numpy(draw_uniforms(args.n2v_walks * (args.L - 1), gen)).to(dev)
    res['node2vec_counted'] = w.count_replay_traffic(st, u)
    if args.dw_walks:
        res['deepwalk'] = rate(DeepWalk(csr, args.L, device=dev), args.dw_walks, args.L, dev)
        res['deepwalk_csr'] = rate(DeepWalk(csr, args.L, device=dev, layout='csr'), args.dw_walks,
                                   args.L, dev)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
