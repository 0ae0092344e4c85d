"""Walker rates on one GPU: DeepWalk and node2vec (p=.25, q=4) walks/s on the device-built R-MAT
graph at several batch sizes (the latency-bound walker needs many walkers in flight; a batch
smaller than the resident capacity leaves CUs idle, one slightly larger pays a whole extra
round). Usage: python scripts/microbench/walk_rates.py [--scale 20] [--edges 10000000]"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'deepwalk-and-node2vec_amd'), REPO]

import torch  # noqa: E402

from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--scale', type=int, default=20)
    ap.add_argument('--edges', type=int, default=10_000_000)
    ap.add_argument('--L', type=int, default=80)
    ap.add_argument('--counts', default='65536,262144,1048576')
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    csr = rmat_graph(args.scale, args.edges, 0, device=dev)
    csr.device_tensors(dev, need_sorted=True)
    N = csr.vocab_size - 1
    t0 = time.perf_counter()
    csr.device_tensors(dev, need_edges=True, need_adj=True)
    torch.cuda.synchronize()
    dd = csr.device_tensors(dev)
    print(f'edge-inline CSR + adjacency hash built in {time.perf_counter() - t0:.3f} s '
          f'({dd["edges"].numel() * 4 / 2**20:.0f} + {dd["adj_hash"].numel() * 4 / 2**20:.0f} MiB)',
          flush=True)
    ref = {}
    for name, mk in (('dw-indexed', lambda: DeepWalk(csr, args.L, rng='philox', seed=7, device=dev)),
                     ('dw-csr', lambda: DeepWalk(csr, args.L, rng='philox', seed=7, device=dev,
                                                 layout='csr')),
                     ('n2v-indexed', lambda: Node2Vec(csr, args.L, p=0.25, q=4.0, rng='philox',
                                                     seed=7, device=dev)),
                     ('n2v-csr', lambda: Node2Vec(csr, args.L, p=0.25, q=4.0, rng='philox',
                                                  seed=7, device=dev, layout='csr'))):
        w = mk()
        for n in (int(c) for c in args.counts.split(',')):
            st = (torch.arange(n, dtype=torch.int64, device=dev) % N + 1).to(torch.int32)
            out = torch.empty((n, args.L), dtype=torch.int32, device=dev)
            w.walk_batch(st[:1024], walk_id0=0, out=out[:1024], check=False)
            torch.cuda.synchronize()
            best = None
            for _ in range(args.reps):
                a = time.perf_counter()
                w.walk_batch(st, walk_id0=0, out=out, check=True)
                torch.cuda.synchronize()
                dt = time.perf_counter() - a
                best = dt if best is None else min(best, dt)
            key = (name.split('-')[0], n)   # both layouts give the same walks
            if key in ref:
                assert torch.equal(ref[key], out), 'inline and csr walks differ'
            else:
                ref[key] = out.clone()
            print(f'{name:11s} n={n:8d}  {best * 1e3:8.2f} ms  {n / best:.3e} walks/s  '
                  f'{n * (args.L - 1) / best:.3e} steps/s', flush=True)
            del out


if __name__ == '__main__':
    main()
