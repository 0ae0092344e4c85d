"""Host enqueue time vs GPU time of the owner-lazy step at C3's 64-walk batch (one GPU).

Prints the mean host time to enqueue one step (no synchronisation inside the loop) and the
mean wall time per step including the final synchronisation: a step is host-bound when the two
agree."""
import sys
import time

import torch

sys.path.insert(0, 'deepwalk-and-node2vec_amd')
from shallow_encoders.graph.random_walk_generator import DeepWalk  # noqa: E402
from shallow_encoders.graph.rmat import rmat_graph  # noqa: E402
from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    csr = rmat_graph(20, 10_000_000, 0, device=dev)
    V = csr.vocab_size
    L, R, K, d, B = 80, 5, 5, 128, 64
    walker = DeepWalk(csr, L, rng='philox', seed=1234, device=dev)
    t = OwnerLazyTables(V, d, dev, lr=0.01, init_seed=0, emulate_world=1, lazy_out=True)
    acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    starts = torch.arange(1, V, dtype=torch.int32, device=dev)
    walks = torch.empty((B, L), dtype=torch.int32, device=dev)
    per = L - 2 * R
    scale = 1.0 / (B * per * 2 * R)

    def step(s):
        walker.walk_batch(starts[(s * B) % (V - 1 - B):][:B], walk_id0=s * B, out=walks,
                          check=False)
        owner_lazy_step(t, walks, R, K, seed=99, noise_offset=s * B * per, grad_scale=scale,
                        loss_acc=acc, status=status)
    for s in range(20):
        step(s)
    torch.cuda.synchronize()
    n = 300
    a = time.perf_counter()
    for s in range(20, 20 + n):
        step(s)
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    print(f'host enqueue {1e3 * (b - a) / n:.3f} ms/step, wall {1e3 * (c - a) / n:.3f} ms/step')


if __name__ == '__main__':
    main()
