"""Device MT19937 stream (dw_mt_uniforms) rates and the end-to-end bit-exact DeepWalk replay at C3.

    python scripts/microbench/mt_rates.py [--stride S]   (S: windows per chain; default: auto)

Prints one JSON line per size: HIP-event time of the generation alone (min of reps), and for
1M C3 walks the end-to-end walk_batch time from the global generator's state.
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

from shallow_encoders.graph import rng as rng_mod  # noqa: E402
from shallow_encoders.graph.random_walk_generator import DeepWalk  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--stride', type=int, default=0)
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    if args.stride:
        rng_mod.mt_window_stride = lambda n, index, n_cu: args.stride
    dev = torch.device('cuda', 0)
    gen = random.Random(1)
    for n in (10_000, 1_000_000, 5_177_344, 82_837_504):
        out = torch.empty(n, dtype=torch.float64, device=dev)
        rng_mod.draw_uniforms_device(n, dev, rng=gen, out=out)
        best = None
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rng_mod.draw_uniforms_device(n, dev, rng=gen, out=out, defer=True)[1]()
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        print(json.dumps({'n': n, 'gen_ms': best, 'GBps': n * 8 / best / 1e6,
                          'stride': rng_mod.mt_window_stride(n, 0, 256)}), flush=True)
    csr = rmat_graph(20, 10_000_000, 0, device=dev)
    csr.device_tensors(dev)
    L, n = 80, 1_048_576
    w = DeepWalk(csr, L, device=dev)
    st = torch.arange(1, n + 1, dtype=torch.int32, device=dev)
    out = torch.empty((n, L), dtype=torch.int32, device=dev)
    random.seed(0)
    w.walk_batch(st, out=out)
    best = None
    for _ in range(args.reps):
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        w.walk_batch(st, out=out)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - a
        best = dt if best is None else min(best, dt)
    print(json.dumps({'deepwalk_replay_walks': n, 'end_to_end_ms': best * 1e3,
                      'walks_per_s': n / best}), flush=True)


if __name__ == '__main__':
    main()
