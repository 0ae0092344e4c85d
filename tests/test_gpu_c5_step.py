"""BASELINE C5 at its own scale: R-MAT 24 (16,777,216 nodes, 256M edge draws), d = 256, node2vec
p = .25, q = 4 (Philox walker), K = 5, R = 5, 8,192 walks of L = 80 per step.

The step runs as bench.py runs C5 on one GPU: sharding.owner_lazy_step on one rank
(OwnerLazyTables(emulate_world=1): the in table's Adam lazy and exact — only the batch's centre
rows are read and updated, their deferred g = 0 steps replayed first — and the out table's dense
Adam fused into the records gather, k_adam_rest covering the rows no record touched).

Checked, per step, from the state the product held before it (as tests/test_gpu_c3_step.py
does at C3), against the reference chain restated by the oracle:
  * walks: every consecutive pair is an edge of the graph (a sorted key set built with torch),
    no walk aborted; the graph's index space needs 64-bit addressing (2E = 513M entries, the
    adjacency hash > 2 GiB);
  * loss terms: oracle.sgns_ref.sgns_coefs_torch in float64 (loss.py:14-22), rtol 1e-5; metric
    counts up to the |logit| < 2^-21 band;
  * gradients, Adam moments and parameters: the float64 closed form (trainer.py:131-152) a
    32-column slab at a time (sgns_grad_columns_torch: the tables are 17 GB each, too large for a
    float64 copy), then torch.optim.Adam(foreach=False) (config_parser/core.py:43-53) on the same
    slab of the same state — the in table on the step's distinct centre rows (their deferred
    g = 0 steps replayed by torch.optim.Adam first), the out table on EVERY row (dense Adam:
    rows no record touched take the g = 0 step). Bars as at C3: gradient (step 1, m / (1 - b1))
    rtol 1e-5, atol 2e-6 max|g|; m rtol 1e-5; v rtol 1e-4; parameters rtol 1e-5 / atol 1e-6 on
    every entry; update p1 - p0 rtol 1e-3 with the gradient atol carried through Adam;
  * the in table's other rows: bit-identical before and after (their step is deferred), their
    step counter unchanged; after the last step a flush brings a sample of lagging rows current,
    equal to torch.optim.Adam's g = 0 steps.
"""
import math

import numpy as np
import pytest
import torch

from oracle import philox as ph
from oracle import sgns_ref

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

SCALE, EDGES = 24, 256_000_000
L, R, K, D, LR, SEED, WALK_SEED, WPN = 80, 5, 5, 256, 0.01, 99, 1234, 10
P, Q = 0.25, 4.0
B = 8192
BETAS, EPS = (0.9, 0.999), 1e-8
STEPS = 3          # step 3 replays deferred steps of rows touched in step 1 only
SLAB = 32          # gradient columns per float64 slab


@pytest.fixture(scope='module')
def c5(hip_device):
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    from shallow_encoders.graph.rmat import rmat_graph
    csr = rmat_graph(SCALE, EDGES, 0, device=hip_device)
    walker = Node2Vec(csr, L, p=P, q=Q, rng='philox', seed=WALK_SEED, device=hip_device)
    yield csr, walker
    import gc
    del csr, walker
    gc.collect()
    torch.cuda.empty_cache()


def _walks(csr, walker, s, dev):
    """Step s's batch as bench.py forms it: global walk ids s*B.., start = id // 10 + 1."""
    g0 = s * B
    n_total = (csr.vocab_size - 1) * WPN
    ids = (torch.arange(g0, g0 + B, device=dev, dtype=torch.int64) % n_total) // WPN + 1
    return walker.walk_batch(ids.to(torch.int32), walk_id0=g0, check=True), g0


def test_c5_walks_are_graph_walks(c5, hip_device):
    dev = hip_device
    csr, walker = c5
    V = csr.vocab_size
    assert V == (1 << SCALE) + 1
    d = csr.device_tensors(dev, need_adj=True)
    row_ptr, col = d['row_ptr'], d['col']
    nnz = int(row_ptr[-1])
    assert row_ptr.dtype == torch.int64 and nnz == csr.nnz and nnz > 500_000_000
    # the walker's adjacency hash spans more than 2 GiB: its probes use 64-bit offsets
    assert int(d['adj_off'][-1]) * 4 > 2 ** 31
    walks = torch.cat([_walks(csr, walker, s, dev)[0] for s in range(STEPS)])
    assert walks.shape == (STEPS * B, L) and bool((walks >= 1).all())
    shift = 1 << 25                                      # V < 2^25: (row, col) in one int64
    rows = torch.repeat_interleave(torch.arange(V, device=dev), row_ptr[1:] - row_ptr[:-1])
    keys = rows.mul_(shift).add_(col.long())
    del rows
    keys, _ = torch.sort(keys)
    q = walks[:, :-1].long() * shift + walks[:, 1:].long()
    pos = torch.searchsorted(keys, q).clamp_(max=nnz - 1)
    ok = keys[pos] == q
    assert bool(ok.all()), f'{int((~ok).sum())} walk steps are not edges'
    # the walks reach the hubs (the p/q step's adjacency tests at large degree)
    deg = (row_ptr[1:] - row_ptr[:-1])[walks.long()]
    print(f'C5 walks: {walks.numel()} nodes, max degree visited {int(deg.max())}, '
          f'{int((deg > 10_000).sum())} visits to nodes of degree > 10K')
    assert int(deg.max()) > 10_000
    del keys, pos, q, ok, deg
    torch.cuda.empty_cache()


def _close(name, got, exp, rtol, atol):
    err = (got.double() - exp.double()).abs()
    lim = atol + rtol * exp.double().abs()
    bad = err > lim
    n_bad = int(bad.sum())
    worst = float((err / lim).max())
    assert n_bad == 0, f'{name}: {n_bad} of {got.numel()} entries outside rtol {rtol} / ' \
                       f'atol {atol:.3e} (worst err/limit {worst:.2f})'
    return worst


def _adam(p, g, m, v, k):
    """torch.optim.Adam(foreach=False) step k on (p, m, v) with gradient g (the reference's
    optimizer); returns (p, m, v) after it."""
    p = p.clone().requires_grad_()
    opt = torch.optim.Adam([p], lr=LR, betas=BETAS, eps=EPS, foreach=False)
    if k > 1:
        opt.state[p] = {'step': torch.tensor(float(k - 1)), 'exp_avg': m.clone(),
                        'exp_avg_sq': v.clone()}
    p.grad = g
    opt.step()
    st = opt.state[p]
    return p.detach(), st['exp_avg'], st['exp_avg_sq']


def _catch_up(p, m, v, last, upto):
    """The reference's g = 0 steps last+1 .. upto on each row (dense Adam updates every row every
    step; the product defers them)."""
    p, m, v = p.clone(), m.clone(), v.clone()
    lo = int(last.min()) + 1 if last.numel() else upto + 1
    for k in range(lo, upto + 1):
        sel = torch.nonzero(last < k).view(-1)
        if sel.numel():
            p[sel], m[sel], v[sel] = _adam(p[sel], torch.zeros_like(p[sel]), m[sel], v[sel], k)
    return p, m, v


def _row_hash(t, chunk=1 << 20):
    """Per-row int64 fingerprint of a float32 [n, d] tensor (bit patterns, position-weighted)."""
    n, d = t.shape
    w = torch.arange(1, d + 1, device=t.device, dtype=torch.int64) * 2654435761
    out = torch.empty(n, dtype=torch.int64, device=t.device)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        out[a:b] = (t[a:b].view(torch.int32).long() * w).sum(1)
    return out


def test_c5_step_full_size_vs_float64_reference(c5, hip_device):
    from shallow_encoders import _native
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    dev = hip_device
    csr, walker = c5
    V = csr.vocab_size
    t = OwnerLazyTables(V, D, dev, lr=LR, betas=BETAS, eps=EPS, init_seed=None, emulate_world=1,
                        lazy_out=False)
    assert t.world == 1 and not t.lazy_out and t.can_fuse_out_adam() and t.V_pad == V
    a = math.sqrt(6.0 / (V + D))                          # W2VBase's Xavier range
    gen = torch.Generator(device=dev).manual_seed(0)
    t.params_in[0, :V].uniform_(-a, a, generator=gen)
    t.w_out[:V].uniform_(-a, a, generator=gen)
    loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    centres = B * (L - 2 * R)
    M = centres * 2 * R
    b1, b2 = BETAS
    w1 = float(np.float32(1 - b1))
    for s in range(STEPS):
        k = s + 1                                        # the Adam step this training step applies
        walks, g0 = _walks(csr, walker, s, dev)
        ins, tgt = sgns_ref.sg_windows_torch(walks, R)
        noise = ph.device_noise_torch(SEED, g0 * (L - 2 * R), centres, 2 * R, K, V, device=dev)
        U = torch.unique(ins)
        n_u = U.numel()
        index = torch.full((V,), -1, dtype=torch.int64, device=dev)
        index[U] = torch.arange(n_u, device=dev)
        # ---- the product's state before the step ---------------------------------------------
        p_in = t.params_in[0]
        last0 = t.last_in[U].clone()
        assert int(last0.max()) <= s
        ref_in0 = _catch_up(p_in[U], t.m_in[U], t.v_in[U], last0, s)   # current to step s
        others = torch.ones(V, dtype=torch.bool, device=dev)
        others[U] = False
        h0 = [_row_hash(x[:V])[others] for x in (p_in, t.m_in, t.v_in)]
        last_others0 = t.last_in[:V][others].clone()
        p_out0, m_out0, v_out0 = t.w_out[:V].clone(), t.m_out[:V].clone(), t.v_out[:V].clone()
        torch.cuda.synchronize()
        loss_acc.zero_()
        owner_lazy_step(t, walks, R, K, seed=SEED, noise_offset=g0 * (L - 2 * R),
                        grad_scale=1.0 / M, loss_acc=loss_acc, status=status)
        torch.cuda.synchronize()
        _native.check_status(status, 'C5 step')
        # ---- rows the step did not touch: deferred, bit-identical -------------------------------
        for name, x, h in zip(('p', 'm', 'v'), (p_in, t.m_in, t.v_in), h0):
            assert bool((_row_hash(x[:V])[others] == h).all()), f'untouched in rows moved ({name})'
        assert bool((t.last_in[:V][others] == last_others0).all())
        assert bool((t.last_in[U] == k).all())
        del h0, last_others0, others
        # ---- the reference step ------------------------------------------------------------
        w_in_c = ref_in0[0]                              # touched rows, current to step s
        ins_c = index[ins]
        sums, ds, dt, band = sgns_ref.sgns_coefs_torch(w_in_c, p_out0, ins_c, tgt, noise)
        print(f'[C5] step {k}: {n_u} distinct centres; loss '
              f'{float(loss_acc[0] + loss_acc[1]) / M:.7f} vs float64 '
              f'{float(sums[0] + sums[1]) / M:.7f}')
        np.testing.assert_allclose(loss_acc[:2].cpu().numpy() / M, sums[:2].cpu().numpy() / M,
                                   rtol=1e-5)
        diff = (loss_acc[2:] - sums[2:]).abs().cpu().numpy()
        assert (diff <= band.cpu().numpy() + 1e-6 * M).all(), (diff, band)
        ident = torch.arange(n_u, device=dev)
        slabs = [(c0, min(D, c0 + SLAB)) for c0 in range(0, D, SLAB)]
        gmax_in = gmax_out = 0.0
        for c0, c1 in slabs:                             # max|g| of each table (the atol scale)
            gi, go = sgns_ref.sgns_grad_columns_torch(w_in_c, p_out0, ins_c, tgt, noise, ds, dt,
                                                      c0, c1, ident, n_u)
            gmax_in = max(gmax_in, float(gi.abs().max()))
            gmax_out = max(gmax_out, float(go.abs().max()))
            del gi, go
        worst = {}
        for c0, c1 in slabs:
            gi, go = sgns_ref.sgns_grad_columns_torch(w_in_c, p_out0, ins_c, tgt, noise, ds, dt,
                                                      c0, c1, ident, n_u)
            for tab, g, gmax, p0, m0, v0, p1, m1, v1 in (
                    ('in', gi, gmax_in, ref_in0[0][:, c0:c1], ref_in0[1][:, c0:c1],
                     ref_in0[2][:, c0:c1], p_in[U, c0:c1], t.m_in[U, c0:c1], t.v_in[U, c0:c1]),
                    ('out', go, gmax_out, p_out0[:, c0:c1], m_out0[:, c0:c1], v_out0[:, c0:c1],
                     t.w_out[:V, c0:c1], t.m_out[:V, c0:c1], t.v_out[:V, c0:c1])):
                g_atol = 2e-6 * gmax
                pr, mr, vr = _adam(p0.contiguous(), g.float(), m0.contiguous(), v0.contiguous(), k)
                res = {}
                if s == 0:        # m0 = 0: m1 = fl((1 - b1) g)
                    res['g'] = _close(f'g_{tab}', m1.double() / w1, g, 1e-5, g_atol)
                res['m'] = _close(f'm_{tab}', m1, mr, 1e-5, (1 - b1) * g_atol)
                res['v'] = _close(f'v_{tab}', v1, vr, 1e-4,
                                  (1 - b2) * (2 * gmax + g_atol) * g_atol)
                res['p'] = _close(f'p_{tab}', p1, pr, 1e-5, 1e-6)
                dp_atol = 1e-8 + LR / (1 - b1 ** k) * (1 - b1) * g_atol / EPS
                res['dp'] = _close(f'dp_{tab}', p1.double() - p0.double(),
                                   pr.double() - p0.double(), 1e-3, dp_atol)
                for q_, w_ in res.items():
                    worst[f'{q_}_{tab}'] = max(worst.get(f'{q_}_{tab}', 0.0), w_)
                del pr, mr, vr
            del gi, go
        print(f'  worst err/limit over all slabs: '
              + ', '.join(f'{q_} {w_:.3f}' for q_, w_ in sorted(worst.items())))
        del p_out0, m_out0, v_out0, ref_in0, ds, dt, noise, index, ins_c, w_in_c
        torch.cuda.empty_cache()
    # ---- after the last step: flush the deferred steps, against torch's g = 0 steps -------------
    lag = torch.nonzero(t.last_in[:V] < STEPS).view(-1)
    lag = lag[(t.last_in[lag] > 0)]                      # rows whose moments are non-zero
    assert lag.numel() > 0
    sample = lag[torch.randperm(lag.numel(), device=dev)[:200_000]]
    exp = _catch_up(t.params_in[0][sample], t.m_in[sample], t.v_in[sample], t.last_in[sample],
                    STEPS)
    t.flush()
    torch.cuda.synchronize()
    for name, got, e in zip(('p', 'm', 'v'), (t.params_in[0][sample], t.m_in[sample],
                                              t.v_in[sample]), exp):
        _close(f'flush_{name}', got, e, 1e-5, 1e-12 if name != 'p' else 1e-6)
    print(f'  flush: {lag.numel()} lagging rows with state, {sample.numel()} checked')
