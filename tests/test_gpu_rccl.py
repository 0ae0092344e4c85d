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
from test_gpu_dist import D, LR, STEPS, run as dist_run, walks_all, V
from test_gpu_owner import (D2, K2, L2, LR2, NW2, R2, STEPS2, V2, _lazy_vs_dense, _walks_all)
from test_gpu_sgns import assert_no_row_drift

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
        from shallow_encoders.word2vec.sharding import OwnerTables, ShardedTables, owner_step
        out = {}
        for mode, pieces in (('overlap', None), ('pieces', 7)):
            t = ShardedTables(V, D, 'cuda:0', lr=LR, init_seed=4, out_pieces=pieces)
            assert t.multi and t.grad_shard is not None and not t.overlap_in
            out[f'sharded_{mode}'] = dist_run(t, walks_all(), 0, 1, mode)
        t = OwnerTables(V2, D2, 'cuda:0', lr=LR2, init_seed=4)
        assert t.multi and t.grad_shard is not None
        per = L2 - 2 * R2
        acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
        status = torch.zeros(1, dtype=torch.int32, device='cuda:0')
        walks = _walks_all()
        for s in range(STEPS2):
            owner_step(t, walks[s].cuda(), R2, K2, seed=11, noise_offset=s * NW2 * per,
                       grad_scale=1.0 / (NW2 * per * 2 * R2), loss_acc=acc, status=status)
        torch.cuda.synchronize()
        _native.check_status(status, 'owner_step')
        out['owner'] = (t.w_in.cpu().numpy().copy(), t.full_w_out().cpu().numpy(),
                        acc.cpu().numpy())
        tl, accl = _lazy_vs_dense('cuda:0', _walks_all(), V2, D2, R2, K2, LR2)
        assert tl.multi
        out['owner_lazy'] = (tl.w_in.cpu().numpy().copy(), tl.full_w_out().cpu().numpy(),
                             accl.cpu().numpy())
        dist.barrier()
        dist.destroy_process_group()
        q.put((out, None))
    except Exception as e:  # report, the parent asserts
        q.put((None, repr(e)))


@pytest.mark.timeout(600)
def test_rccl_one_rank_protocols_equal_single_process(hip_device):
    from shallow_encoders.word2vec.sharding import ShardedTables
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    p = ctx.Process(target=_child, args=(_free_port(), q))
    p.start()
    res, err = q.get(timeout=500)
    p.join(timeout=60)
    assert err is None, err
    assert p.exitcode == 0

    # replicated layout: vs the serial one-device step over the same batches
    ref = ShardedTables(V, D, hip_device, lr=LR, init_seed=4)
    ri, ro = dist_run(ref, walks_all(), 0, 1, 'serial')
    for mode in ('overlap', 'pieces'):
        gi, go = res[f'sharded_{mode}']
        for got, exp in ((gi, ri), (go, ro)):
            bad = ~np.isclose(got, exp, rtol=1e-4, atol=1e-6)
            assert bad.mean() < 1e-3, (mode, bad.mean())
            assert np.abs(got - exp).max() <= 2.05 * LR * STEPS

    # owner layouts: vs single-process dense training
    ref = ShardedTables(V2, D2, hip_device, lr=LR2, init_seed=4)
    walks = _walks_all()
    per = L2 - 2 * R2
    acc_ref = torch.zeros(4, dtype=torch.float64, device=hip_device)
    for s in range(STEPS2):
        sgns_accumulate(ref.w_in, ref.w_out, ref.g_in, ref.g_out, K2, walks=walks[s].cuda(),
                        context_radius=R2, seed=11, noise_offset=s * NW2 * per,
                        loss_acc=acc_ref)
        ref.step()
    torch.cuda.synchronize()
    for key in ('owner', 'owner_lazy'):
        wi, wo, acc = res[key]
        np.testing.assert_allclose(acc, acc_ref.cpu().numpy(), rtol=1e-5, atol=1e-6)
        for got, exp in ((wi, ref.w_in.cpu().numpy()), (wo, ref.w_out.cpu().numpy())):
            bad = ~np.isclose(got, exp, rtol=1e-4, atol=1e-6)
            assert bad.mean() < 1e-3, (key, bad.mean())
            assert_no_row_drift(got, exp, rtol=1e-4)
            assert np.abs(got - exp).max() <= 2.05 * LR2 * STEPS2
