"""The overlapped multi-rank step on a real GPU: 2 ranks (gloo, both on cuda:0) drive
dw_sgns_walks_phase + ShardedTables.exchange_in / exchange_out / sync with the HIP Adam.

This exercises the side-stream ordering: the in-table reduce-scatter / Adam / all-gather is
issued after pass 1 while pass 2 still reads the old in table from the other buffer. After a
few steps both replicas must equal a single-process run (world 1, serial step) over the whole
batch. The 'pieces' form runs the output-table phase in row pieces (sgns_phase2_pieces ->
dw_sgns_walks_phase2_piece) with each piece exchanged on the side stream behind the next
piece's gather (ShardedTables.exchange_out_piece), as bench.py does at N > 1. The RCCL variant
of the same code runs in bench.py at N > 1; RCCL refuses two ranks on one device, so gloo
carries the collectives here.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

V, D, R, K, L, NW, STEPS, LR = 600, 64, 2, 3, 12, 64, 3, 1e-3


def walks_all():
    g = torch.Generator().manual_seed(5)
    return torch.randint(1, V, (STEPS, NW, L), generator=g, dtype=torch.int32)


def sharded_snapshot(tables):
    """(w_in, w_out, m[0], v[0], m[1], v[1], rows[0], rows[1]) of this rank (numpy): the
    replicated tables and this rank's Adam rows with their global row ids."""
    return (tables.w_in.cpu().numpy().copy(), tables.w_out.cpu().numpy().copy(),
            tables.m[0].cpu().numpy().copy(), tables.v[0].cpu().numpy().copy(),
            tables.m[1].cpu().numpy().copy(), tables.v[1].cpu().numpy().copy(),
            tables.state_rows(0).numpy(), tables.state_rows(1).numpy())


def assemble(per_rank_snaps, V_pad, V):
    """Full (V, d) tables + Adam state per step from every rank's sharded snapshots."""
    out = []
    for step in zip(*per_rank_snaps):
        w_in, w_out = step[0][0], step[0][1]
        d = w_in.shape[1]
        full = [np.zeros((V_pad, d), np.float32) for _ in range(4)]
        for sn in step:
            for k, (t, rows) in enumerate(((2, 6), (3, 6), (4, 7), (5, 7))):
                full[k][sn[rows]] = sn[t]
        out.append((w_in, w_out) + tuple(f[:V] for f in full))
    return out


def init_tables():
    from shallow_encoders.word2vec.sharding import ShardedTables
    t = ShardedTables(V, D, 'cpu', lr=LR, init_seed=4)
    return t.w_in.numpy().copy(), t.w_out.numpy().copy()


def run(tables, walks, rank, world, mode, snaps=None):
    """mode: 'serial' | 'overlap' | 'pieces'. ``snaps``: a list receiving sharded_snapshot after
    every step."""
    from shallow_encoders.word2vec.sgns import sgns_accumulate, sgns_phase2_pieces
    dev = tables.device
    per = L - 2 * R
    scale = 1.0 / (NW * per * 2 * R)
    half = NW // world
    for s in range(STEPS):
        w = walks[s, rank * half:(rank + 1) * half].to(dev)
        kw = dict(walks=w, context_radius=R, seed=11, noise_offset=s * NW * per + rank * half * per,
                  grad_scale=scale)
        if mode != 'serial':
            sgns_accumulate(tables.w_in, tables.w_out, tables.g_in, tables.g_out, K, phase=1, **kw)
            tables.exchange_in()
            if mode == 'pieces':
                n_pieces, rows = tables.out_pieces_spec()
                sgns_phase2_pieces(tables.w_in, tables.g_out, K, walks=w, context_radius=R,
                                   n_pieces=n_pieces, piece_rows=rows,
                                   on_piece=tables.exchange_out_piece)
            else:
                sgns_accumulate(tables.w_in, tables.w_out, tables.g_in, tables.g_out, K,
                                phase=2, **kw)
            tables.exchange_out()
            tables.sync()
        else:
            sgns_accumulate(tables.w_in, tables.w_out, tables.g_in, tables.g_out, K, **kw)
            tables.step()
        if snaps is not None:
            torch.cuda.synchronize(dev)
            snaps.append(sharded_snapshot(tables))
    torch.cuda.synchronize(dev)
    return tables.w_in.cpu().numpy().copy(), tables.w_out.cpu().numpy().copy()


def _worker(rank, world, port, mode, pieces, q):
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from shallow_encoders.word2vec.sharding import ShardedTables
        t = ShardedTables(V, D, 'cuda:0', lr=LR, init_seed=4, out_pieces=pieces)
        snaps = []
        wi, wo = run(t, walks_all(), rank, world, mode, snaps)
        q.put((rank, wi, wo, (snaps, t.V_pad), None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report, the parent asserts
        q.put((rank, None, None, None, repr(e)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.timeout(600)
@pytest.mark.parametrize('mode,pieces', [('overlap', None), ('pieces', None), ('pieces', 7)])
def test_overlapped_exchange_two_ranks_equals_single_process(hip_device, mode, pieces):
    """Both replicas identical after every all-gather, and EVERY step of the 2-rank run equal
    to the reference step from the state before it (tests/stepcheck.py: float64 closed-form
    gradient of the global batch + torch.optim.Adam; the single-step bars, no fraction
    allowance)."""
    from stepcheck import check_trajectory
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, pieces, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=500) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[4] for r in res if r[4]]
    assert not errs, errs
    (_, i0, o0, (s0, V_pad), _), (_, i1, o1, (s1, _), _) = res
    np.testing.assert_array_equal(i0, i1)
    np.testing.assert_array_equal(o0, o1)
    for a, b in zip(s0, s1):                      # replicas identical after every step
        np.testing.assert_array_equal(a[0], b[0])
        np.testing.assert_array_equal(a[1], b[1])
    worst = check_trajectory(f'2 ranks {mode}', init_tables(), assemble([s0, s1], V_pad, V),
                             walks_all(), R, K, 11, LR, NW * (L - 2 * R))
    print({k: round(v, 3) for k, v in sorted(worst.items())})
