"""The N>1 owner-computes protocol (OwnerTables: out table sharded by row owner o % world, no
output-table collective; in table replicated with a node-range reduce-scatter / Adam /
all-gather) with world_size 2 and 3 over gloo on the CPU.

Every rank sees the whole global batch and contributes the gradient of the output slots whose
row it owns (oracle.sgns_ref.sgns_grads_closed_form(owner=...), the restatement of what
dw_sgns_owner_pass1/_pass2 compute on the GPU). After several steps the in-table replicas and
the gathered out table must equal single-process training on the whole batch, and every row's
Adam state must exist exactly once.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sgns_ref
from test_dist_gloo import V, D, R, K, STEPS, batches, cpu_adam


def owner_train(t, rank, world):
    rows = t.out_rows().numpy()
    keep = rows < t.V
    for ins, tgt, noise in batches():
        _, gi, go = sgns_ref.sgns_grads_closed_form(t.w_in.numpy(), t.full_w_out().numpy(), ins,
                                                    tgt, noise, owner=rank, n_owners=world)
        # rows this rank does not own get no gradient from its slots
        foreign = np.ones(V, bool)
        foreign[rows[keep]] = False
        assert np.abs(go[foreign]).max(initial=0.0) == 0.0
        w_in_before = t.w_in.clone()
        t.g_in.add_(torch.as_tensor(gi, dtype=torch.float32))      # pass 1 (partial g_in)
        t.exchange_in()
        assert torch.equal(t.w_in, w_in_before)   # the output-table phase sees the old in table
        t.g_out[keep] += torch.as_tensor(go[rows[keep]], dtype=torch.float32)   # pass 2
        t.out_step()
        t.sync()
        assert float(t.grads_in.abs().max()) == 0.0 and float(t.g_out.abs().max()) == 0.0


def _worker(rank, world, port, q, force=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if force:   # one rank that still runs the N > 1 protocol with its collectives
        os.environ['DW_FORCE_COLLECTIVES'] = '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from shallow_encoders.word2vec.sharding import OwnerTables
    t = OwnerTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    assert t.multi == (world > 1 or force)
    owner_train(t, rank, world)
    m_out, v_out = t.out_state_full()
    q.put((rank, t.w_in.numpy().copy(), t.full_w_out().numpy(), t.shard_range(),
           t.m_in.numpy().copy(), m_out.numpy(), t.out_rows().numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_owner_split_sums_to_full_gradient():
    """The oracle's owner split is a partition of the slots: the parts add up to the whole."""
    from test_dist_gloo import batches as b
    rng = np.random.default_rng(1)
    w_in, w_out = rng.normal(size=(V, D)), rng.normal(size=(V, D))
    ins, tgt, noise = b()[0]
    loss, gi, go = sgns_ref.sgns_grads_closed_form(w_in, w_out, ins, tgt, noise)
    for world in (2, 3, 8):
        parts = [sgns_ref.sgns_grads_closed_form(w_in, w_out, ins, tgt, noise, owner=r,
                                                 n_owners=world) for r in range(world)]
        np.testing.assert_allclose(sum(p[0] for p in parts), loss, rtol=1e-12)
        np.testing.assert_allclose(sum(p[1] for p in parts), gi, rtol=1e-10, atol=1e-14)
        np.testing.assert_allclose(sum(p[2] for p in parts), go, rtol=1e-10, atol=1e-14)


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world,force', [(2, False), (3, False), (1, True)])
def test_owner_tables_equal_single_process(world, force):
    from shallow_encoders.word2vec.sharding import ShardedTables
    from test_dist_gloo import train
    ref = ShardedTables(V, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    train(ref, 0, 1, 'serial')
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, force)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        np.testing.assert_array_equal(res[0][1], res[r][1])   # replicas identical
        np.testing.assert_array_equal(res[0][2], res[r][2])
    np.testing.assert_allclose(res[0][1], ref.w_in.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res[0][2], ref.w_out.numpy(), rtol=1e-5, atol=1e-6)
    # in-table Adam state: node-id ranges; out-table: every row in exactly one slice
    S = res[0][3][1] - res[0][3][0]
    assert [r[3] for r in res] == [(k * S, (k + 1) * S) for k in range(world)]
    m_in = np.concatenate([r[4] for r in res])[:V]
    np.testing.assert_allclose(m_in, ref.m[0].numpy()[:V], rtol=1e-4, atol=1e-9)
    owned = np.concatenate([r[6] for r in res])
    assert sorted(owned.tolist()) == list(range(S * world))
    np.testing.assert_allclose(res[0][5], ref.m[1].numpy()[:V], rtol=1e-4, atol=1e-9)


# ---- the touched-row in-table exchange (OwnerLazyTables) -------------------------------------
# sparse batches over a larger vocabulary: most rows miss several steps, so the deferred Adam
# updates are replayed (catch_up / flush) rather than applied every step
VL, NWL, LL, STEPS_L = 300, 4, 9, 5


def lazy_batches():
    rng = np.random.default_rng(7)
    out = []
    for _ in range(STEPS_L):
        walks = rng.integers(1, VL, size=(NWL, LL))
        ins, tgt = sgns_ref.sg_windows(walks, R)
        noise = rng.integers(0, VL, size=(len(ins), 2 * R, K))
        out.append((ins, tgt, noise))
    return out


def lazy_train(t, rank, world):
    rows = t.out_rows().numpy()
    keep = rows < t.V
    for ins, tgt, noise in lazy_batches():
        U = np.unique(ins.reshape(-1))
        t.begin_step()
        t.set_touched(torch.as_tensor(U))
        t.catch_up()
        _, gi, go = sgns_ref.sgns_grads_closed_form(t.w_in_raw.numpy(), t.full_w_out().numpy(),
                                                    ins, tgt, noise, owner=rank, n_owners=world)
        untouched = np.setdiff1d(np.arange(t.V), U)
        assert np.abs(gi[untouched]).max(initial=0.0) == 0.0   # only centres get a gradient
        t.g_in.add_(torch.as_tensor(gi, dtype=torch.float32))
        t.exchange_touched()
        t.g_out[keep] += torch.as_tensor(go[rows[keep]], dtype=torch.float32)
        t.out_step()
        t.update_touched()
        assert float(t.grads_in.abs().max()) == 0.0
        # rows outside U lag behind: the deferral is really exercised
        assert int(t.last_in[torch.as_tensor(untouched)].min()) < t.step_count or t.step_count == 1


def _lazy_worker(rank, world, port, q, force=False):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    if force:
        os.environ['DW_FORCE_COLLECTIVES'] = '1'
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from shallow_encoders.word2vec.sharding import OwnerLazyTables
    t = OwnerLazyTables(VL, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    assert t.multi == (world > 1 or force)
    lazy_train(t, rank, world)
    w_in = t.w_in.numpy().copy()             # flushes every deferred update
    assert int(t.last_in.min()) == t.step_count
    q.put((rank, w_in, t.full_w_out().numpy(), t.m_in.numpy().copy(), t.v_in.numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world,force', [(1, False), (2, False), (3, False), (1, True)])
def test_owner_lazy_tables_equal_dense_single_process(world, force):
    from shallow_encoders.word2vec.sharding import ShardedTables
    ref = ShardedTables(VL, D, 'cpu', lr=0.05, init_seed=3, adam_impl=cpu_adam)
    for ins, tgt, noise in lazy_batches():
        _, gi, go = sgns_ref.sgns_grads_closed_form(ref.w_in.numpy(), ref.w_out.numpy(), ins, tgt,
                                                    noise)
        ref.g_in.add_(torch.as_tensor(gi, dtype=torch.float32))
        ref.g_out.add_(torch.as_tensor(go, dtype=torch.float32))
        ref.step()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lazy_worker, args=(r, world, port, q, force))
             for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(1, world):
        np.testing.assert_array_equal(res[0][1], res[r][1])   # replicas identical
        np.testing.assert_array_equal(res[0][3], res[r][3])
    np.testing.assert_allclose(res[0][1], ref.w_in.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(res[0][2], ref.w_out.numpy(), rtol=1e-5, atol=1e-6)
    # the replicated in-table Adam state after the flush equals the dense optimizer's
    np.testing.assert_allclose(res[0][3][:VL], ref.m[0].numpy()[:VL], rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(res[0][4][:VL], ref.v[0].numpy()[:VL], rtol=1e-4, atol=1e-12)
