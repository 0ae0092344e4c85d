"""The small-batch step replayed as a HIP graph (word2vec/graphed.py) equals the eager step.

C2's shape (a 4,096-node R-MAT with Cora's edge count, node2vec p=1 q=1, L=10, R=2, K=5, d=128,
64-walk batches): the same walks bit for bit, the same negatives and Adam steps, so the losses
agree to float64-atomic order and the tables to fp32 atomic-order noise (the bars of
test_gpu_sgns.py: at most 0.1% of entries outside rtol 1e-5 / atol 1e-6, none by more than
lr / 100, no row drifting as a whole)."""
import numpy as np
import pytest
import torch

from test_gpu_sgns import assert_no_row_drift, assert_params_close

pytestmark = pytest.mark.gpu

B, L, R, K, D, LR, WPN, SEED = 64, 10, 2, 5, 128, 0.01, 16, 99


def _setup(dev):
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    from shallow_encoders.graph.rmat import rmat_graph
    from shallow_encoders.word2vec.graphed import epoch_starts_node_order
    csr = rmat_graph(12, 5429, 0, device=dev)
    walker = Node2Vec(csr, L, p=1.0, q=1.0, rng='philox', seed=1234, device=dev)
    starts = epoch_starts_node_order(csr.vocab_size - 1, WPN, dev)
    return csr, walker, starts


@pytest.mark.parametrize('scatter,overlap_in,unroll', [('sorted', True, 1), ('atomic', True, 1),
                                                       ('atomic', False, 1), ('sorted', True, 3),
                                                       ('atomic', False, 4)])
def test_graphed_step_equals_eager(hip_device, scatter, overlap_in, unroll):
    """overlap_in=False: both tables' Adam in one in-place launch after pass 1 (bench.py's tiny
    atomic-scatter graphs), one captured graph instead of one per in-table buffer. unroll > 1:
    several steps per graph (an odd unroll flips the in-table buffer, so two graphs)."""
    from shallow_encoders.word2vec.graphed import GraphedStep
    from shallow_encoders.word2vec.sharding import ShardedTables, replicated_step
    dev = hip_device
    csr, walker, epoch = _setup(dev)
    V = csr.vocab_size
    grad_scale = 1.0 / (B * (L - 2 * R) * 2 * R)
    warm, steps = 2, 12
    runs = []
    for mode in ('eager', 'graph'):
        t = ShardedTables(V, D, dev, lr=LR, init_seed=0, overlap_in=overlap_in)
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)

        def eager(s):
            g0 = s * B
            st = epoch[torch.arange(g0, g0 + B, device=dev) % epoch.numel()]
            walks = walker.walk_batch(st, walk_id0=g0, check=False)
            replicated_step(t, walks, R, K, seed=SEED, noise_offset=g0 * (L - 2 * R),
                            grad_scale=grad_scale, loss_acc=acc, status=status, scatter=scatter,
                            fuse_out_adam=scatter == 'sorted')
            return walks
        for s in range(warm):                   # allocates the workspaces, as bench.py does
            eager(s)
        if mode == 'eager':
            for s in range(warm, warm + steps):
                last = eager(s)
        else:
            gs = GraphedStep(t, walker, epoch, B, R, K, seed=SEED, grad_scale=grad_scale,
                             loss_acc=acc, status=status, first_walk_id=warm * B,
                             n_steps=steps, scatter=scatter, unroll=unroll)
            for _ in range(steps // unroll):
                gs.replay()
            last = gs.walks[-B:]          # the last step of the last graph
            sc = gs.scalars()
            assert sc == {'walk_id0': (warm + steps) * B,
                          'noise_offset': (warm + steps) * B * (L - 2 * R),
                          'step': warm + steps + 1}
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        assert t.step_count == warm + steps
        runs.append((t.w_in.cpu().numpy(), t.w_out.cpu().numpy(), acc.cpu().numpy(),
                     last.cpu().numpy()))
    (wi_e, wo_e, acc_e, walks_e), (wi_g, wo_g, acc_g, walks_g) = runs
    np.testing.assert_array_equal(walks_g, walks_e)        # same walk ids and starts
    # the loss sums are float64 atomics over tables that already differ by fp32 atomic-order
    # noise (below): a run measured 1.05e-9 relative on the 12-step positive-loss sum
    np.testing.assert_allclose(acc_g, acc_e, rtol=1e-8 if scatter == 'atomic' else 1e-9)
    # the atomic scatter sums every out-row gradient in a run-dependent order, so each of the 12
    # Adam steps can amplify an ulp in any near-zero gradient entry (not only at chunk edges as
    # the sorted path): a run measured 1.06e-4 on one entry against lr/100; lr/10 there
    lim = LR / 10 if scatter == 'atomic' else None
    for got, exp in ((wi_g, wi_e), (wo_g, wo_e)):
        assert_params_close(got, exp, LR, max_abs=lim)
        assert_no_row_drift(got, exp)


@pytest.mark.parametrize('lazy_out,unroll,late', [(True, 1, False), (True, 4, False),
                                                  (False, 3, False), (True, 12, False),
                                                  (True, 4, True)])
def test_graphed_owner_lazy_step_equals_eager(hip_device, lazy_out, unroll, late, monkeypatch):
    """The one-GPU lazy owner step (bench.py's path for the reference's 64-walk batch on a large
    graph) replayed as a HIP graph (GraphedOwnerStep: the lazy kernels' step numbers bound
    relative to the step blocks) equals the eager steps: the same walks, losses to float64-atomic
    order, and both tables, flushed, to fp32 atomic-order noise. late: the side-first capture
    (the next step's preparation enqueued before the out rows) replayed from the first step."""
    from shallow_encoders.word2vec import graphed as graphed_mod
    from shallow_encoders.word2vec.graphed import GraphedOwnerStep
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    if late:
        monkeypatch.setattr(graphed_mod, 'SIDE_FIRST_FROM', 0)
    dev = hip_device
    csr, walker, epoch = _setup(dev)
    V = csr.vocab_size
    grad_scale = 1.0 / (B * (L - 2 * R) * 2 * R)
    warm, steps = 2, 12
    runs = []
    for mode in ('eager', 'graph'):
        t = OwnerLazyTables(V, D, dev, lr=LR, init_seed=0, emulate_world=1, lazy_out=lazy_out)
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)

        def eager(s):
            g0 = s * B
            st = epoch[torch.arange(g0, g0 + B, device=dev) % epoch.numel()]
            walks = walker.walk_batch(st, walk_id0=g0, check=False)
            owner_lazy_step(t, walks, R, K, seed=SEED, noise_offset=g0 * (L - 2 * R),
                            grad_scale=grad_scale, loss_acc=acc, status=status)
            return walks
        for s in range(warm):
            eager(s)
        if mode == 'eager':
            for s in range(warm, warm + steps):
                last = eager(s)
        else:
            gs = GraphedOwnerStep(t, walker, epoch, B, R, K, seed=SEED, grad_scale=grad_scale,
                                  loss_acc=acc, status=status, first_walk_id=warm * B,
                                  n_steps=steps, unroll=unroll)
            for _ in range(steps // unroll):
                gs.replay()
            last = gs.walks[-B:]
            sc = gs.scalars()
            assert sc == {'walk_id0': (warm + steps) * B,
                          'noise_offset': (warm + steps) * B * (L - 2 * R),
                          'step': warm + steps + 1}
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        assert t.step_count == warm + steps
        t._flush_out()          # (an emulated one-rank slice is the whole out table)
        runs.append((t.w_in.cpu().numpy(), t.w_out[:V].cpu().numpy(), acc.cpu().numpy(),
                     last.cpu().numpy()))
    (wi_e, wo_e, acc_e, walks_e), (wi_g, wo_g, acc_g, walks_g) = runs
    np.testing.assert_array_equal(walks_g, walks_e)
    # float64 atomic loss sums over tables with fp32 atomic-order noise: measured 1.03e-9
    np.testing.assert_allclose(acc_g, acc_e, rtol=1e-8)
    # a row's records are summed in the order the claim's atomics ranked them, which differs
    # between the two runs, and 12 Adam steps can amplify an ulp of a near-zero gradient entry:
    # a run measured 1.4e-4 on one entry against lr/100; lr/10 there (the atomic scatter's bar)
    for got, exp in ((wi_g, wi_e), (wo_g, wo_e)):
        assert_params_close(got, exp, LR, max_abs=LR / 10)
        assert_no_row_drift(got, exp)


@pytest.mark.parametrize('n_steps', [1, 2, 7])
def test_pipelined_owner_steps_equal_sequential(hip_device, n_steps):
    """owner_lazy_steps (step k + 1's claims, touch claim and catch-up on side streams while
    step k runs) equals the sequential owner_lazy_step calls on the same batches: the small
    graph's batches share most centre rows from step to step, so the catch-up of step k + 1 must
    skip exactly the centres step k updates. Losses to float64-atomic order, tables to fp32
    atomic-order noise; and the pipelined run leaves the tables ready for an eager step."""
    from shallow_encoders.word2vec.sharding import (OwnerLazyTables, owner_lazy_step,
                                                    owner_lazy_steps)
    dev = hip_device
    csr, walker, epoch = _setup(dev)
    V = csr.vocab_size
    grad_scale = 1.0 / (B * (L - 2 * R) * 2 * R)
    warm = 2
    batches = []
    for s in range(warm + n_steps + 1):
        g0 = s * B
        st = epoch[torch.arange(g0, g0 + B, device=dev) % epoch.numel()]
        batches.append((walker.walk_batch(st, walk_id0=g0, check=False), g0 * (L - 2 * R)))
    runs = []
    for mode in ('sequential', 'pipelined'):
        t = OwnerLazyTables(V, D, dev, lr=LR, init_seed=0, emulate_world=1, lazy_out=True)
        assert t.pipeline_ok(R, K)
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)

        def one(k):
            owner_lazy_step(t, batches[k][0], R, K, seed=SEED, noise_offset=batches[k][1],
                            grad_scale=grad_scale, loss_acc=acc, status=status)
        for k in range(warm):
            one(k)
        run = range(warm, warm + n_steps)
        if mode == 'sequential':
            for k in run:
                one(k)
        else:
            owner_lazy_steps(t, [batches[k][0] for k in run], R, K, seed=SEED,
                             noise_offsets=[batches[k][1] for k in run],
                             grad_scale=grad_scale, loss_acc=acc, status=status)
        one(warm + n_steps)     # an eager step after the run
        torch.cuda.synchronize()
        assert int(status.item()) == 0
        assert t.step_count == warm + n_steps + 1
        t._flush_out()
        runs.append((t.w_in.cpu().numpy(), t.w_out[:V].cpu().numpy(), acc.cpu().numpy()))
    (wi_s, wo_s, acc_s), (wi_p, wo_p, acc_p) = runs
    np.testing.assert_allclose(acc_p, acc_s, rtol=1e-8)
    for got, exp in ((wi_p, wi_s), (wo_p, wo_s)):
        assert_params_close(got, exp, LR, max_abs=LR / 10)
        assert_no_row_drift(got, exp)


def test_lazy_kernels_refuse_a_block_bound_without_its_step(hip_device):
    """dw_adam_rows (and the other lazy launches) take step numbers relative to a block bound by
    dw_step_scalars_bind_at; under a plain dw_step_scalars_bind they refuse instead of capturing
    a frozen step."""
    from shallow_encoders import _native
    from shallow_encoders.word2vec.sharding import hip_rows_adam
    dev = hip_device
    p = torch.zeros((4, 64), device=dev)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    last = torch.zeros(4, dtype=torch.int32, device=dev)
    hist = torch.zeros((8, 8), device=dev)
    blk = torch.zeros(64, dtype=torch.uint8, device=dev)
    _native.call('dw_step_scalars_bind', _native.ptr(blk))
    try:
        with pytest.raises(Exception, match='bind_at'):
            hip_rows_adam(p, m, v, last, None, None, 4, None, hist, 1)
    finally:
        _native.call('dw_step_scalars_bind', None)
