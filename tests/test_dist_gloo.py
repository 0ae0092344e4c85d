"""The N>1 exchange (node-id-range sharded Adam: reduce-scatter -> Adam on own rows ->
all-gather, per table) with world_size 2 over gloo on the CPU.

Two ranks each take half of the batch (DDP semantics: local gradient scaled by 1/M_global);
after several steps their replicated tables must equal single-process training on the whole
batch. Both forms are checked: the serial ``step()`` and the overlapped protocol bench.py uses
(``exchange_in`` after pass 1 -> output-table gradient computed from ``w_in`` -> ``exchange_out``
-> ``sync``), where the in-table update must land in the second buffer so the output-table
phase still sees the old in table. The 'pieces' form hands the output-table gradient over in
row pieces, each exchanged (exchange_out_piece) before the next piece's rows are added, as
bench.py does at N > 1 behind dw_sgns_walks_phase2_piece; it also runs with a piece count that
does not divide the vocabulary (padding rows). The gradient and Adam math here is the
oracle's (CPU); on the GPU the same ShardedTables object drives dw_sgns_walks_phase +
dw_adam_dense over RCCL.
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
    """mode: 'serial' | 'overlap' | 'pieces'."""
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
            if mode == 'pieces':
                n_pieces, rows = t.out_pieces_spec()
                for p in range(n_pieces):        # pass 2, piece by piece
                    a, b = p * rows, min((p + 1) * rows, t.V)
                    w_out_before = t.w_out[a:b].clone()
                    if a < b:
                        t.g_out[a:b].add_(go[a:b])
                    t.exchange_out_piece(p)
                    if world > 1 and a < b:
                        assert not torch.equal(t.w_out[a:b], w_out_before)  # piece updated
            else:
                t.g_out.add_(go)                 # pass 2
            t.exchange_out()
            t.sync()
        assert float(t.grads.abs().max()) == 0.0


def _worker(rank, world, port, mode, pieces, q, force=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if force:   # one rank that still runs the N > 1 protocol with its collectives
        os.environ['DW_FORCE_COLLECTIVES'] = '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from shallow_encoders.word2vec.sharding import ShardedTables
    t = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam, out_pieces=pieces)
    assert t.multi == (world > 1 or force)
    train(t, rank, world, mode)
    q.put((rank, t.w_in.numpy().copy(), t.w_out.numpy().copy(),
           (t.shard_range(), t.P, t.S, t.V_pad),
           [(t.state_rows(k).numpy(), t.m[k].numpy().copy()) for k in (0, 1)]))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(300)
@pytest.mark.parametrize('mode,pieces', [('serial', None), ('overlap', None), ('serial', 3),
                                         ('pieces', None), ('pieces', 3)])
def test_sharded_adam_world2_equals_single_process(mode, pieces):
    from shallow_encoders.word2vec.sharding import ShardedTables
    ref = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    assert ref.world == 1
    train(ref, 0, 1, 'serial')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, pieces, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, i0, o0, g0, st0), (_, i1, o1, g1, st1) = res
    np.testing.assert_array_equal(i0, i1)                 # replicas identical after all-gather
    np.testing.assert_array_equal(o0, o1)
    (r0, P, S, V_pad), (r1, _, _, _) = g0, g1
    assert P == (pieces or 8) and V_pad % (2 * P) == 0 and V_pad >= V
    assert r0 == (0, S) and r1 == (S, 2 * S)              # node-id ranges of the in table
    np.testing.assert_allclose(i0, ref.w_in.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o0, ref.w_out.numpy(), rtol=1e-5, atol=1e-6)
    for k in (0, 1):                                      # Adam state, by global row
        rows = np.concatenate([st0[k][0], st1[k][0]])
        m = np.concatenate([st0[k][1], st1[k][1]])
        assert sorted(rows.tolist()) == list(range(V_pad))   # every row owned exactly once
        keep = rows < V
        np.testing.assert_allclose(m[keep][np.argsort(rows[keep])], ref.m[k].numpy(),
                                   rtol=1e-4, atol=1e-9)


@pytest.mark.timeout(300)
@pytest.mark.parametrize('mode,pieces', [('serial', None), ('pieces', 3)])
def test_sharded_forced_collectives_one_rank_equals_single_process(mode, pieces):
    """DW_FORCE_COLLECTIVES=1 at world 1 (how tests/test_gpu_rccl.py and bench.py's
    DW_BENCH_DIST=1 run the RCCL flow on one GPU): the N > 1 protocol, reduce-scatter /
    all-gather included, over a one-rank group equals the one-device step."""
    from shallow_encoders.word2vec.sharding import ShardedTables
    ref = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    train(ref, 0, 1, 'serial')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(0, 1, _free_port(), mode, pieces, q, True))
    p.start()
    _, i0, o0, (r0, P, S, V_pad), _ = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert P == (pieces or 8) and r0 == (0, V_pad) and S == V_pad
    np.testing.assert_allclose(i0, ref.w_in.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(o0, ref.w_out.numpy(), rtol=1e-5, atol=1e-6)
