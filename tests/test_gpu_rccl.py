"""The multi-GPU step's RCCL flow on a one-GPU box: one rank in a real 'nccl' (RCCL) process
group with DW_FORCE_COLLECTIVES=1, so the N > 1 protocols run with their collectives instead of
the one-device shortcuts:
- ShardedTables (replicated layout, §7.2): reduce-scatter of g_in / g_out pieces, Adam on the
  own rows, in-place all-gather, all on the side stream behind the output-table phase;
- OwnerTables (owner-computes, sharded in table, §7.1): reduce-scatter + all-gather of the in
  table on the side stream, the out slice's Adam fused into pass 2, full_w_out's all-gather;
- OwnerLazyTables (touched-row exchange): the |U| readback and the all-reduce of the touched
  rows' gradient on the side stream, waited on by the current stream.

RCCL refuses two ranks on one device, so the two-rank tests (test_gpu_dist.py,
test_gpu_owner.py) carry their collectives over gloo; this file is what runs the same code over
RCCL itself (the backend bench.py uses at N > 1): the calls are accepted (shapes, in-place
all-gather, async work handles waited on from another stream) and a one-rank job equals the
single-process result. Sequences that must match across ranks are covered by the gloo tests.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from shallow_encoders import _native
from shallow_encoders.word2vec.sgns import sgns_accumulate
from stepcheck import check_trajectory
from test_gpu_dist import (D, K, L, LR, NW, R, assemble, init_tables, run as dist_run,
                           walks_all, V)
from test_gpu_owner import D2, K2, L2, LR2, NW2, R2, STEPS2, V2, _walks_all

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child(port, q):
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        os.environ['DW_FORCE_COLLECTIVES'] = '1'
        torch.cuda.set_device(0)
        dist.init_process_group('nccl', rank=0, world_size=1,
                                device_id=torch.device('cuda', 0))
        assert dist.get_backend() == 'nccl'
        from shallow_encoders.word2vec.sharding import (OwnerLazyTables, OwnerTables,
                                                        ShardedTables, owner_lazy_step,
                                                        owner_step)
        out = {}
        for mode, pieces in (('overlap', None), ('pieces', 7)):
            t = ShardedTables(V, D, 'cuda:0', lr=LR, init_seed=4, out_pieces=pieces)
            assert t.multi and t.grad_shard is not None and not t.overlap_in
            snaps = []
            dist_run(t, walks_all(), 0, 1, mode, snaps)
            out[f'sharded_{mode}'] = assemble([snaps], t.V_pad, V)
        per = L2 - 2 * R2
        status = torch.zeros(1, dtype=torch.int32, device='cuda:0')
        walks = _walks_all()

        def owner_snap(t):
            return (t.w_in.cpu().numpy().copy(), t.full_w_out().cpu().numpy(),
                    t.m_in[:V2].cpu().numpy().copy(), t.v_in[:V2].cpu().numpy().copy(),
                    t.m_out[:V2].cpu().numpy().copy(), t.v_out[:V2].cpu().numpy().copy())

        t = OwnerTables(V2, D2, 'cuda:0', lr=LR2, init_seed=4)
        assert t.multi and t.grad_shard is not None
        acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
        snaps = []
        for s in range(STEPS2):
            owner_step(t, walks[s].cuda(), R2, K2, seed=11, noise_offset=s * NW2 * per,
                       grad_scale=1.0 / (NW2 * per * 2 * R2), loss_acc=acc, status=status)
            torch.cuda.synchronize()
            snaps.append(owner_snap(t))
        _native.check_status(status, 'owner_step')
        out['owner'] = (snaps, acc.cpu().numpy())
        for lazy_out in (False, True):
            tl = OwnerLazyTables(V2, D2, 'cuda:0', lr=LR2, init_seed=4, lazy_out=lazy_out)
            assert tl.multi
            acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
            snaps = []
            for s in range(STEPS2):
                # sparse batches: a quarter of the walks, so rows lag between steps
                w = walks[s][:NW2 // 4].cuda()
                owner_lazy_step(tl, w, R2, K2, seed=11, noise_offset=s * (NW2 // 4) * per,
                                grad_scale=1.0 / ((NW2 // 4) * per * 2 * R2), loss_acc=acc,
                                status=status)
                torch.cuda.synchronize()
                # the state with every deferred step applied, the tables left lagging
                lag = [tl.params_in, tl.m_in, tl.v_in, tl.last_in]
                if tl.lazy_out:
                    lag += [tl.w_out, tl.m_out, tl.v_out, tl.last_out, tl.pend_out]
                keep = [x.clone() for x in lag]
                tl.flush()
                snaps.append(owner_snap(tl))
                for dst, src in zip(lag, keep):
                    dst.copy_(src)
            _native.check_status(status, 'owner_lazy_step')
            out[f'owner_lazy_{int(lazy_out)}'] = (snaps, acc.cpu().numpy())
        dist.barrier()
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:  # report, the parent asserts
        q.put((None, repr(e)))


@pytest.mark.timeout(600)
def test_rccl_one_rank_protocols_equal_single_process(hip_device):
    """Every step of every protocol, run over RCCL, equals the reference step from the state
    before it (tests/stepcheck.py: float64 closed-form gradient + torch.optim.Adam, the
    single-step bars with no fraction allowance)."""
    from shallow_encoders.word2vec.sharding import ShardedTables
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    res, err = q.get(timeout=500)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0
    per = L - 2 * R
    for mode in ('overlap', 'pieces'):
        worst = check_trajectory(f'rccl sharded {mode}', init_tables(), res[f'sharded_{mode}'],
                                 walks_all(), R, K, 11, LR, NW * per)
        print(mode, {k: round(v, 3) for k, v in sorted(worst.items())})
    t0 = ShardedTables(V2, D2, 'cpu', lr=LR2, init_seed=4)
    init2 = (t0.w_in.numpy().copy(), t0.w_out.numpy().copy())
    per2 = L2 - 2 * R2
    walks = _walks_all()
    for key, nw in (('owner', NW2), ('owner_lazy_0', NW2 // 4), ('owner_lazy_1', NW2 // 4)):
        snaps, acc = res[key]
        worst = check_trajectory(f'rccl {key}', init2, snaps, walks[:, :nw], R2, K2, 11, LR2,
                                 nw * per2)
        print(key, {k: round(v, 3) for k, v in sorted(worst.items())})
    # the loss sums of the whole run against single-process dense training
    ref = ShardedTables(V2, D2, hip_device, lr=LR2, init_seed=4)
    acc_ref = torch.zeros(4, dtype=torch.float64, device=hip_device)
    for s in range(STEPS2):
        sgns_accumulate(ref.w_in, ref.w_out, ref.g_in, ref.g_out, K2, walks=walks[s].cuda(),
                        context_radius=R2, seed=11, noise_offset=s * NW2 * per2,
                        loss_acc=acc_ref)
        ref.step()
    torch.cuda.synchronize()
    np.testing.assert_allclose(res['owner'][1], acc_ref.cpu().numpy(), rtol=1e-5, atol=1e-6)
