"""The benchmarked C3 step at its full size, against an independent float64 reference.

bench.py's headline step (R-MAT 20: V = 1,048,577; d = 128; 8,192 Philox DeepWalk walks of L = 80;
R = 5, K = 5 device negatives; lr 0.01) runs here exactly as the bench composes it:

  * 'dense' (the N = 1 default, sharding.replicated_step): SGNS pass 1 -> in-table Adam out of
    place on a side stream with its grid capped to 47 blocks (dw_adam_dense_to) || records sort
    + gather with the out-table Adam fused (dw_sgns_walks_phase2_adam, k_adam_rest) -> join;
  * 'lazy' (the one-GPU default at C5, sharding.owner_lazy_step on one rank): the owner passes
    with the touched-row exact Adam of the in table, deferred g = 0 steps replayed.

Each step is checked from the state the product held before it (tables and Adam moments),
against the reference chain restated by the oracle, not against another product path:
  * negatives: oracle.philox.device_noise_torch (the counter layout, pinned on CPU against the
    numpy restatement);
  * windows: sg_windows_torch (W2VCollateFunctional order, torch_dataset.py:293-322);
  * loss, g_in, g_out: sgns_grads_closed_form_torch, float64 (loss.py:14-22 + the autograd
    gradient of the batch mean, trainer.py:131-152);
  * update: torch.optim.Adam(foreach=False) (the reference's optimizer, config_parser/core.py:43-53)
    on the same state, given the float64 gradient rounded to float32.

Stated tolerances (fp32 kernels vs the float64 reference):
  * loss terms: rtol 1e-5; metric counts (recall / precision) equal up to the terms with
    |logit| < 2^-21, where a float32 sigmoid may round to exactly .5 either way;
  * gradient (step 1, read back as m / (1 - beta1) because the fused step never materialises it):
    rtol 1e-5, atol 2e-6 x max|g| (tests/test_gpu_sgns.py assert_grad_close);
  * Adam moments: m rtol 1e-5 + (1 - beta1) x the gradient atol; v rtol 1e-4 + its square term;
  * parameters: EVERY entry within rtol 1e-5, atol 1e-6 (SURVEY.md §8c single-step bar; no
    fraction allowance, so no row can drift), and the update p1 - p0 within rtol 1e-3 and an
    atol of 1e-8 + the gradient atol carried through Adam: (lr / bc1)(1 - beta1) g_atol / eps.
"""
import numpy as np
import pytest
import torch

from oracle import philox as ph
from oracle import sgns_ref

pytestmark = pytest.mark.gpu

SCALE, EDGES = 20, 10_000_000
L, R, K, D, LR, SEED, WALK_SEED, WPN = 80, 5, 5, 128, 0.01, 99, 1234, 10
BETAS, EPS = (0.9, 0.999), 1e-8


@pytest.fixture(scope='module')
def c3(hip_device):
    from shallow_encoders.graph.random_walk_generator import DeepWalk
    from shallow_encoders.graph.rmat import rmat_graph
    csr = rmat_graph(SCALE, EDGES, 0, device=hip_device)
    csr.device_tensors(hip_device)
    walker = DeepWalk(csr, L, rng='philox', seed=WALK_SEED, device=hip_device)
    return csr, walker


def _walks(csr, walker, s, dev, B):
    """Step s's batch as bench.py forms it: global walk ids s*B.., start = id // 10 + 1."""
    g0 = s * B
    n_total = (csr.vocab_size - 1) * WPN
    ids = (torch.arange(g0, g0 + B, device=dev, dtype=torch.int64) % n_total) // WPN + 1
    return walker.walk_batch(ids.to(torch.int32), walk_id0=g0, check=True), g0


class _Dense:
    def __init__(self, V, dev):
        from shallow_encoders.word2vec.sharding import ShardedTables
        self.t = ShardedTables(V, D, dev, lr=LR, betas=BETAS, eps=EPS, init_seed=0)
        assert self.t.overlap_in and self.t.can_fuse_out_adam()
        self.V = V

    def state(self):
        t, V = self.t, self.V
        return (t.w_in, t.w_out, t.m[0, :V], t.v[0, :V], t.m[1, :V], t.v[1, :V])

    def snapshot(self):
        return [x.clone() for x in self.state()]

    def step(self, walks, g0, loss_acc, status):
        from shallow_encoders.word2vec.sharding import replicated_step
        centres = walks.shape[0] * (L - 2 * R)
        replicated_step(self.t, walks, R, K, seed=SEED, noise_offset=g0 * (L - 2 * R),
                        grad_scale=1.0 / (centres * 2 * R), loss_acc=loss_acc, status=status)


class _Lazy:
    def __init__(self, V, dev, lazy_out=False):
        from shallow_encoders.word2vec.sharding import OwnerLazyTables
        self.t = OwnerLazyTables(V, D, dev, lr=LR, betas=BETAS, eps=EPS, init_seed=0,
                                 emulate_world=1, lazy_out=lazy_out)
        assert self.t.lazy_out == lazy_out
        self.V = V

    def state(self):
        t, V = self.t, self.V
        t.flush()            # the deferred g = 0 steps, replayed exactly
        return (t.params_in[0, :V], t.w_out[:V], t.m_in[:V], t.v_in[:V], t.m_out[:V],
                t.v_out[:V])

    def snapshot(self):
        """The current state with every deferred step applied, leaving the tables as they were
        (rows outside the next batch keep lagging, so the step's catch-up is exercised)."""
        t = self.t
        lagging = [t.params_in, t.m_in, t.v_in, t.last_in]
        if t.lazy_out:
            lagging += [t.w_out, t.m_out, t.v_out, t.last_out, t.pend_out]
        keep = [x.clone() for x in lagging]
        dirty = t._pend_dirty
        snap = [x.clone() for x in self.state()]
        for dst, src in zip(lagging, keep):
            dst.copy_(src)
        t._pend_dirty = dirty
        return snap

    def step(self, walks, g0, loss_acc, status):
        from shallow_encoders.word2vec.sharding import owner_lazy_step
        centres = walks.shape[0] * (L - 2 * R)
        owner_lazy_step(self.t, walks, R, K, seed=SEED, noise_offset=g0 * (L - 2 * R),
                        grad_scale=1.0 / (centres * 2 * R), loss_acc=loss_acc, status=status)


def _close(name, got, exp, rtol, atol):
    err = (got - exp).abs()
    lim = atol + rtol * exp.abs()
    bad = err > lim
    n_bad = int(bad.sum())
    worst = float((err / lim).max())
    print(f'  {name}: max|err| {float(err.max()):.3e}, worst err/limit {worst:.3f}')
    assert n_bad == 0, f'{name}: {n_bad} of {got.numel()} entries outside rtol {rtol} / ' \
                       f'atol {atol:.3e} (worst err/limit {worst:.2f})'


@pytest.mark.parametrize('composition,B,steps', [('dense', 8192, 3), ('lazy', 8192, 3),
                                                 ('lazy_out', 64, 6)])
def test_c3_step_full_size_vs_float64_reference(c3, composition, B, steps, hip_device):
    """'lazy_out': the reference's 64-walk batch on the full C3 tables, both tables' Adam lazy
    (a step touches ~23% of the out rows; the others' deferred steps are replayed exactly)."""
    from shallow_encoders import _native
    dev = hip_device
    csr, walker = c3
    V = csr.vocab_size
    assert V == 1_048_577
    prod = (_Dense(V, dev) if composition == 'dense' else
            _Lazy(V, dev, lazy_out=composition == 'lazy_out'))
    loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    centres = B * (L - 2 * R)
    M = centres * 2 * R
    b1, b2 = BETAS
    w1 = np.float32(1 - b1)
    for s in range(steps):
        walks, g0 = _walks(csr, walker, s, dev, B)
        p_in0, p_out0, m_in0, v_in0, m_out0, v_out0 = prod.snapshot()
        torch.cuda.synchronize()
        loss_acc.zero_()
        prod.step(walks, g0, loss_acc, status)
        torch.cuda.synchronize()
        _native.check_status(status, 'C3 step')
        p_in1, p_out1, m_in1, v_in1, m_out1, v_out1 = prod.snapshot()

        # ---- the reference step from the same state ----------------------------------------
        ins, tgt = sgns_ref.sg_windows_torch(walks, R)
        noise = ph.device_noise_torch(SEED, g0 * (L - 2 * R), centres, 2 * R, K, V, device=dev)
        sums, g_in, g_out, band = sgns_ref.sgns_grads_closed_form_torch(p_in0, p_out0, ins, tgt,
                                                                        noise, with_band=True)
        del noise
        print(f'[{composition}] step {s + 1}: loss {float(loss_acc[0] + loss_acc[1]) / M:.7f} '
              f'vs float64 {float(sums[0] + sums[1]) / M:.7f}')
        np.testing.assert_allclose(loss_acc[:2].cpu().numpy() / M, sums[:2].cpu().numpy() / M,
                                   rtol=1e-5)
        # metric counts: equal up to the terms whose fp32 sigmoid may round to exactly .5
        diff = (loss_acc[2:] - sums[2:]).abs().cpu().numpy()
        print(f'  metric counts {loss_acc[2:].tolist()} vs {sums[2:].tolist()}, '
              f'|diff| {diff.tolist()} <= band {band.tolist()}')
        assert (diff <= band.cpu().numpy() + 1e-6 * M).all()
        ref_p = [p_in0.clone().requires_grad_(), p_out0.clone().requires_grad_()]
        opt = torch.optim.Adam(ref_p, lr=LR, betas=BETAS, eps=EPS, foreach=False)
        if s > 0:
            for p, m, v in zip(ref_p, (m_in0, m_out0), (v_in0, v_out0)):
                opt.state[p] = {'step': torch.tensor(float(s)), 'exp_avg': m.clone(),
                                'exp_avg_sq': v.clone()}
        for p, g in zip(ref_p, (g_in, g_out)):
            p.grad = g.to(torch.float32)
        opt.step()
        for tab, g, m0, m1, v1, p0, p1, pr in (
                ('in', g_in, m_in0, m_in1, v_in1, p_in0, p_in1, ref_p[0]),
                ('out', g_out, m_out0, m_out1, v_out1, p_out0, p_out1, ref_p[1])):
            st = opt.state[pr]
            g_atol = 2e-6 * float(g.abs().max())
            if s == 0:   # m0 = 0: m1 = fl((1 - beta1) * g)
                _close(f'g_{tab}', m1.double() / float(w1), g, 1e-5, g_atol)
            _close(f'm_{tab}', m1, st['exp_avg'], 1e-5, (1 - b1) * g_atol)
            _close(f'v_{tab}', v1, st['exp_avg_sq'], 1e-4,
                   (1 - b2) * (2 * float(g.abs().max()) + g_atol) * g_atol)
            _close(f'p_{tab}', p1, pr.detach(), 1e-5, 1e-6)
            # the update's sensitivity to m is at most (lr / bc1) / eps, so the gradient bar
            # carries over as (lr / bc1) * (1 - beta1) * g_atol / eps
            dp_atol = 1e-8 + LR / (1 - b1 ** (s + 1)) * (1 - b1) * g_atol / EPS
            _close(f'dp_{tab}', (p1 - p0).double(), (pr.detach() - p0).double(), 1e-3, dp_atol)
        del ref_p, opt, g_in, g_out
