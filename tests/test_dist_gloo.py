"""The N>1 exchange (node-id-range sharded Adam: reduce-scatter -> Adam on own rows ->
all-gather, per table) with world_size 2 over gloo on the CPU.

Two ranks each take half of the batch (DDP semantics: local gradient scaled by 1/M_global);
after several steps their replicated tables must equal single-process training on the whole
batch. Both forms are checked: the serial ``step()`` and the overlapped protocol bench.py uses
(``exchange_in`` after pass 1 -> output-table gradient computed from ``w_in`` -> ``exchange_out``
-> ``sync``), where the in-table update must land in the second buffer so the output-table
phase still sees the old in table. The gradient and Adam math here is the oracle's (CPU); on
the GPU the same ShardedTables object drives dw_sgns_walks_phase + dw_adam_dense over RCCL.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sgns_ref

V, D, R, K, L, STEPS = 50, 8, 2, 3, 9, 3


def cpu_adam(p, g, m, v, step, lr, betas, eps, wd, zero_grad):
    """torch.optim.Adam's single-tensor update on flat CPU buffers (test stand-in for HIP)."""
    b1, b2 = betas
    if wd:
        g = g + wd * p
    m.lerp_(g, 1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    denom = (v.sqrt() / bc2 ** 0.5).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if zero_grad:
        g.zero_()


def batches():
    rng = np.random.default_rng(0)
    out = []
    for _ in range(STEPS):
        walks = rng.integers(1, V, size=(8, L))
        ins, tgt = sgns_ref.sg_windows(walks, R)
        noise = rng.integers(0, V, size=(len(ins), 2 * R, K))
        out.append((ins, tgt, noise))
    return out


def grads(tables, ins, tgt, noise, share):
    _, gi, go = sgns_ref.sgns_grads_closed_form(tables.w_in.numpy(), tables.w_out.numpy(), ins,
                                                tgt, noise)
    return (torch.as_tensor(gi * share, dtype=torch.float32),
            torch.as_tensor(go * share, dtype=torch.float32))


def train(t, rank, world, mode):
    for ins, tgt, noise in batches():
        half = len(ins) // world
        sl = slice(rank * half, (rank + 1) * half)
        gi, go = grads(t, ins[sl], tgt[sl], noise[sl], 1.0 / world)
        if mode == 'serial':
            t.g_in.add_(gi)
            t.g_out.add_(go)
            t.step()
        else:
            w_in_before = t.w_in.clone()
            t.g_in.add_(gi)                      # pass 1: centre-table gradient final
            t.exchange_in()
            assert torch.equal(t.w_in, w_in_before)  # output-table phase sees the old in table
            t.g_out.add_(go)                     # pass 2
            t.exchange_out()
            t.sync()
        assert float(t.grads.abs().max()) == 0.0


def _worker(rank, world, port, mode, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from shallow_encoders.word2vec.sharding import ShardedTables
    t = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    train(t, rank, world, mode)
    q.put((rank, t.w_in.numpy().copy(), t.w_out.numpy().copy(), t.shard_range(),
           t.m.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
@pytest.mark.parametrize('mode', ['serial', 'overlap'])
def test_sharded_adam_world2_equals_single_process(mode):
    from shallow_encoders.word2vec.sharding import ShardedTables
    ref = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    assert ref.world == 1
    train(ref, 0, 1, 'serial')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, i0, o0, r0, m0), (_, i1, o1, r1, m1) = res
    np.testing.assert_array_equal(i0, i1)                 # replicas identical after all-gather
    np.testing.assert_array_equal(o0, o1)
    assert r0 == (0, V // 2) and r1 == (V // 2, V)        # node-id-range rows of both tables
    np.testing.assert_allclose(i0, ref.w_in.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o0, ref.w_out.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(np.concatenate([m0, m1], axis=1), ref.m.numpy(), rtol=1e-4,
                               atol=1e-9)
