"""Fused SGNS kernel, logits kernels and HIP Adam on the MI355X vs the reference fixtures and
the oracle. fp32 tolerances: loss / gradients rtol 1e-5 (atomic accumulation order differs
from torch's embedding_dense_backward), Adam-updated parameters rtol 1e-5 / atol 1e-6."""
import glob
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from oracle import philox as ph
from oracle import sgns_ref

from shallow_encoders import _native
from shallow_encoders.word2vec.model import SkipGram
from shallow_encoders.word2vec.optim import Adam
from shallow_encoders.word2vec.sgns import SGNSLoss, loss_terms, sgns_accumulate

pytestmark = pytest.mark.gpu

ALL_SGNS = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, 'sgns_*.npz')))
# skip-gram, no max_norm (the records / walks paths); CBOW and max_norm fixtures below
SGNS_FIXTURES = [n for n in ALL_SGNS if 'cbow' not in n and 'maxnorm' not in n]
POOLED_FIXTURES = [n for n in ALL_SGNS if n not in SGNS_FIXTURES]
RTOL = 1e-5          # fp32 gradients / losses
ATOL_REL = 2e-6      # absolute slack, relative to the largest gradient entry (cancellations)


def assert_grad_close(got, exp):
    np.testing.assert_allclose(got, exp, rtol=RTOL, atol=ATOL_REL * float(np.abs(exp).max()))


def assert_params_close(got, exp, lr, rtol=1e-5, atol=1e-6, max_frac=1e-3, max_abs=None):
    """Adam-updated parameters. Adam normalises every gradient entry (m / sqrt(v)), so an entry
    whose gradient is a near-cancelling sum (|g| ~ eps) amplifies the ulp-level difference of
    atomic vs torch accumulation order up to O(lr); such entries are rare. Allowed: at most
    `max_frac` of the entries outside (rtol, atol), and none beyond `max_abs` (lr/100)."""
    bad = ~np.isclose(got, exp, rtol=rtol, atol=atol)
    assert bad.mean() <= max_frac, f'{bad.sum()} / {bad.size} entries outside tolerance'
    lim = lr / 100 if max_abs is None else max_abs
    assert np.abs(got - exp).max() <= lim, (np.abs(got - exp).max(), lim)


def assert_no_row_drift(got, exp, rtol=1e-5, atol=1e-6, max_row_frac=0.25):
    """Adam amplifies accumulation-order noise only in isolated entries (gradients ~0); an extra
    or missing update of a row moves (nearly) all of its entries. No row may have more than
    ``max_row_frac`` of its entries outside (rtol, atol)."""
    bad = ~np.isclose(got, exp, rtol=rtol, atol=atol)
    frac = bad.mean(axis=1)
    rows = np.nonzero(frac > max_row_frac)[0]
    assert rows.size == 0, f'rows drifted as a whole: {rows[:10].tolist()} ({frac[rows[:10]]})'


def reference_envelope(w_in0, w_out0, lr, batches, rtol=1e-5, atol=1e-6):
    """How far the REFERENCE's own trajectory moves when its gradients are summed exactly
    (float64 closed form, rounded to float32) instead of in torch's order: the fp32
    reproducibility envelope of a multi-step lr-scaled Adam run. Returns (frac, max_abs) of
    that trajectory against the reference plus the final tables."""
    ref = sgns_ref.TorchAdamRef(w_in0, w_out0, lr=lr)
    for ins, tgt, noise, *step_lr in batches:
        if step_lr:
            ref.opt.param_groups[0]['lr'] = step_lr[0]
        _, gi, go = sgns_ref.sgns_grads_closed_form(*ref.tables(), ins, tgt, noise)
        ref.step(gi.astype(np.float32), go.astype(np.float32))
    return ref.tables()


def assert_within_envelope(got, exp, exact, lr, rtol=1e-5, atol=1e-6):
    """got (HIP) may deviate from the reference exp at most ~4x as much as the exact-sum
    trajectory does (fraction of entries outside (rtol, atol) and max |diff|)."""
    bad_exact = (~np.isclose(exact, exp, rtol=rtol, atol=atol)).mean()
    max_exact = float(np.abs(exact - exp).max())
    assert_params_close(got, exp, lr, rtol, atol,
                        max_frac=4 * bad_exact + max(1e-3, 2.0 / got.size),
                        max_abs=4 * max_exact + lr / 100)


def _dev(x, dtype=None):
    t = torch.as_tensor(np.ascontiguousarray(x))
    return t.to('cuda', dtype) if dtype is not None else t.cuda()


def _tables(f):
    return _dev(f['w_in0'], torch.float32), _dev(f['w_out0'], torch.float32)


@pytest.mark.parametrize('name', SGNS_FIXTURES)
@pytest.mark.parametrize('mode', ['pairs', 'walks'])
@pytest.mark.parametrize('scatter', ['sorted', 'atomic'])
def test_fused_sgns_step_vs_reference(name, mode, scatter, hip_device):
    f = golden(name)
    w_in, w_out = _tables(f)
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    K, R = int(f['K']), int(f['R'])
    noise = _dev(f['noise'][0], torch.int64)
    if mode == 'pairs':
        acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, inputs=_dev(f['inputs'], torch.int64),
                              targets=_dev(f['targets'], torch.int64), noise=noise,
                              scatter=scatter)
    else:
        acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, walks=_dev(f['walks'], torch.int32),
                              context_radius=R, noise=noise, scatter=scatter)
    t = loss_terms(acc, f['targets'].size, K)
    np.testing.assert_allclose([float(t['loss']), float(t['positive-loss']),
                                float(t['negative-loss'])], f['losses'][0], rtol=1e-5)
    assert float(t['recall']) == pytest.approx(float(f['recall'][0]), abs=1e-6)
    assert float(t['precision']) == pytest.approx(float(f['precision'][0]), abs=1e-6)
    assert_grad_close(g_in.cpu().numpy(), f['g_in'])
    assert_grad_close(g_out.cpu().numpy(), f['g_out'])


@pytest.mark.parametrize('name', SGNS_FIXTURES)
def test_hip_adam_trajectory_vs_reference(name, hip_device):
    """Reference training steps (fixture noise) through fused SGNS + HIP Adam."""
    f = golden(name)
    w_in = torch.nn.Parameter(_dev(f['w_in0'], torch.float32))
    w_out = torch.nn.Parameter(_dev(f['w_out0'], torch.float32))
    opt = Adam([w_in, w_out], lr=float(f['lr']))
    w_in.grad, w_out.grad = torch.zeros_like(w_in), torch.zeros_like(w_out)
    K = int(f['K'])
    inputs, targets = _dev(f['inputs'], torch.int64), _dev(f['targets'], torch.int64)
    for step in range(f['noise'].shape[0]):
        acc = sgns_accumulate(w_in.detach(), w_out.detach(), w_in.grad, w_out.grad, K,
                              inputs=inputs, targets=targets,
                              noise=_dev(f['noise'][step], torch.int64))
        t = loss_terms(acc, f['targets'].size, K)
        assert float(t['loss']) == pytest.approx(float(f['losses'][step][0]), rel=1e-5)
        opt.step()
        assert float(w_in.grad.abs().max()) == 0.0  # fused zero_grad
        lr = float(f['lr'])
        if step == 0:
            ex_in, ex_out = reference_envelope(f['w_in0'], f['w_out0'], lr,
                                               [(f['inputs'], f['targets'], f['noise'][0])])
            assert_within_envelope(w_in.detach().cpu().numpy(), f['w_in1'], ex_in, lr)
            assert_within_envelope(w_out.detach().cpu().numpy(), f['w_out1'], ex_out, lr)
    ex_in, ex_out = reference_envelope(
        f['w_in0'], f['w_out0'], lr,
        [(f['inputs'], f['targets'], f['noise'][s]) for s in range(f['noise'].shape[0])])
    assert_within_envelope(w_in.detach().cpu().numpy(), f['w_in_n'], ex_in, lr)
    assert_within_envelope(w_out.detach().cpu().numpy(), f['w_out_n'], ex_out, lr)


def test_adam_kernel_vs_torch_adam_random_grads(hip_device):
    rng = np.random.default_rng(0)
    n = 1000 * 128 + 3  # tail elements exercise the scalar path
    p0 = rng.standard_normal(n).astype(np.float32)
    p = torch.nn.Parameter(_dev(p0, torch.float32))
    ref = torch.tensor(p0, requires_grad=True)
    opt = Adam([p], lr=0.01, betas=(0.8, 0.99), eps=1e-7, weight_decay=0.01)
    ropt = torch.optim.Adam([ref], lr=0.01, betas=(0.8, 0.99), eps=1e-7, weight_decay=0.01,
                            foreach=False)
    for _ in range(4):
        g = rng.standard_normal(n).astype(np.float32) * 1e-2
        p.grad = _dev(g, torch.float32)
        ref.grad = torch.tensor(g)
        opt.step()
        ropt.step()
    np.testing.assert_allclose(p.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5,
                               atol=1e-6)
    st = opt.state[p]
    np.testing.assert_allclose(st['exp_avg'].cpu().numpy(), ropt.state[ref]['exp_avg'].numpy(),
                               rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(st['exp_avg_sq'].cpu().numpy(),
                               ropt.state[ref]['exp_avg_sq'].numpy(), rtol=1e-5, atol=1e-10)


@pytest.mark.parametrize('n_pieces,extra', [(1, 0), (3, 0), (8, 5), (64, 0), (1024, 0)])
def test_phase2_pieces_equal_phase2(hip_device, n_pieces, extra):
    """dw_sgns_walks_phase2_piece: the sort call then the gathers of n_pieces row pieces (some
    empty, piece_rows over-covering V by `extra` rows per piece) give phase 2's g_out (float
    atomic order aside: chunk boundaries move with the pieces), and each piece call touches
    only its own rows."""
    from shallow_encoders.word2vec.sgns import sgns_phase2_pieces
    g = torch.Generator().manual_seed(n_pieces)
    V, d, R, K, n, L = 3000, 128, 3, 4, 200, 30
    walks = torch.randint(0, V, (n, L), generator=g, dtype=torch.int32)
    walks[:, ::4] = 5                                   # a hub row spanning many chunks
    walks = walks.to(hip_device)
    w_in = (torch.rand((V, d), generator=g) - 0.5).to(hip_device)
    w_out = (torch.rand((V, d), generator=g) - 0.5).to(hip_device)
    kw = dict(walks=walks, context_radius=R, seed=3)
    ref_in, ref_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    sgns_accumulate(w_in, w_out, ref_in, ref_out, K, **kw)
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    sgns_accumulate(w_in, w_out, g_in, g_out, K, phase=1, **kw)
    rows = -(-V // n_pieces) + extra
    seen = []

    def on_piece(p):
        torch.cuda.synchronize()
        done = g_out.abs().sum(dim=1) > 0
        lo, hi = p * rows, min((p + 1) * rows, V)
        assert not bool(done[hi:].any()), f'piece {p} wrote rows of later pieces'
        seen.append(p)

    sgns_phase2_pieces(w_in, g_out, K, walks=walks, context_radius=R, n_pieces=n_pieces,
                       piece_rows=rows, on_piece=on_piece)
    torch.cuda.synchronize()
    assert seen == list(range(n_pieces))
    # (float-atomic order at the hub row's chunk boundaries: thousands of terms summed in a
    # run-dependent order, so the bar scales with the largest entry; 1e-7 of it failed 1 entry
    # in 384,000 at 1.4x the bar on one run)
    np.testing.assert_allclose(g_in.cpu().numpy(), ref_in.cpu().numpy(), rtol=1e-5,
                               atol=1e-6 * float(ref_in.abs().max()))
    np.testing.assert_allclose(g_out.cpu().numpy(), ref_out.cpu().numpy(), rtol=1e-5,
                               atol=1e-6 * float(ref_out.abs().max()))


@pytest.mark.parametrize('max_blocks', [0, 32, 47])
def test_adam_dense_to_equals_in_place(hip_device, max_blocks):
    """dw_adam_dense_to (read one buffer, write another; capped grid-stride grids) is
    bit-identical to the in-place dw_adam_dense and leaves the source untouched; both zero the
    gradient."""
    from shallow_encoders.word2vec.sharding import hip_adam, hip_adam_to
    rng = np.random.default_rng(1)
    n = 4096 * 64 + 7
    p0, g0, m0, v0 = (rng.standard_normal(n).astype(np.float32) for _ in range(4))
    v0 = np.abs(v0)
    a = [_dev(x, torch.float32) for x in (p0, g0, m0, v0)]
    b = [_dev(x, torch.float32) for x in (p0, g0, m0, v0)]
    dst = torch.full_like(b[0], float('nan'))
    hp = (3, 0.01, (0.9, 0.999), 1e-8, 0.01)
    hip_adam(*a, *hp, True)
    hip_adam_to(b[0], dst, b[1], b[2], b[3], *hp, True, max_blocks)
    torch.cuda.synchronize()
    assert torch.equal(dst, a[0])
    assert torch.equal(b[0].cpu(), torch.tensor(p0))
    for x, y in zip(a[1:], b[1:]):
        assert torch.equal(x, y)
    assert float(b[1].abs().max()) == 0.0


@pytest.mark.parametrize('n16', [1, 1023, 1024, 1025, 300_001])
def test_stream_copy_copies_exactly(hip_device, n16):
    """dw_stream_copy (bench.py's measured copy roofline) copies every 16-B lane of ragged sizes
    (a partial last tile) and nothing beyond them."""
    n = n16 * 4
    src = torch.randn(n + 8, device=hip_device)
    dst = torch.full((n + 8,), -7.0, device=hip_device)
    _native.call('dw_stream_copy', _native.ptr(src), _native.ptr(dst), n * 4,
                 _native.stream(hip_device))
    torch.cuda.synchronize()
    assert torch.equal(dst[:n], src[:n])
    assert bool((dst[n:] == -7.0).all())


@pytest.mark.parametrize('fuse', [True, False])
def test_overlapped_in_table_adam_equals_serial(hip_device, fuse):
    """One GPU: the in-table Adam on the side stream into the second buffer (overlap_in) gives
    the tables of the serial in-place update, with and without the fused out-table Adam."""
    from shallow_encoders.graph.random_walk_generator import DeepWalk
    from shallow_encoders.graph.rmat import rmat_graph
    from shallow_encoders.word2vec.sharding import ShardedTables
    csr = rmat_graph(12, 40_000, 0, device=hip_device)
    walker = DeepWalk(csr, 40, rng='philox', seed=3, device=hip_device)
    V, R, K, nw, d = csr.vocab_size, 3, 4, 256, 128
    ov = ShardedTables(V, d, hip_device, lr=0.02, init_seed=5, overlap_in=True)
    se = ShardedTables(V, d, hip_device, lr=0.02, init_seed=5, overlap_in=False)
    assert ov.overlap_in and not se.overlap_in and ov.params.shape[0] == 3
    for step in range(4):
        starts = torch.randint(1, V, (nw,), generator=torch.Generator().manual_seed(step),
                               dtype=torch.int32).to(hip_device)
        walks = walker.walk_batch(starts, walk_id0=step * nw)
        for t in (ov, se):
            kw = dict(walks=walks, context_radius=R, seed=7, noise_offset=step * nw * 34)
            sgns_accumulate(t.w_in, t.w_out, t.g_in, t.g_out, K, phase=1, **kw)
            t.exchange_in()
            spec = t.out_adam_spec() if fuse else None
            sgns_accumulate(t.w_in, t.w_out, t.g_in, t.g_out, K, phase=2, out_adam=spec, **kw)
            t.exchange_out(fused_out=fuse)
            t.sync()
    torch.cuda.synchronize()
    assert ov._cur_in == 0 and float(ov.grads.abs().max()) == 0.0
    for a, b in ((ov.w_in, se.w_in), (ov.w_out, se.w_out)):
        assert_params_close(a.cpu().numpy(), b.cpu().numpy(), 0.02, max_frac=5e-3,
                            max_abs=2.05 * 0.02 * 4)
    # the serial step() path on the 3-slot layout
    ov.step()
    torch.cuda.synchronize()
    assert float(ov.grads.abs().max()) == 0.0


@pytest.mark.parametrize('d,hub', [(100, False), (128, False), (256, False), (300, False),
                                   (128, True), (64, True)])
def test_fused_sgns_random_case_vs_oracle(d, hub, hip_device):
    """Larger vocabularies / masked widths against the torch-CPU oracle (autograd). `hub`:
    every 3rd walk position is node 7, so row 7 collects thousands of records and straddles
    many 512-record chunks of the sorted path (boundary atomics)."""
    rng = np.random.default_rng(d)
    V, R, K, L, n = 20_000, 5, 5, 40, 48
    w_in0, w_out0 = sgns_ref.xavier_tables(V, d, seed=d)
    walks = rng.integers(0, V, size=(n, L)).astype(np.int32)
    if hub:
        walks[:, ::3] = 7
    ins, tgt = sgns_ref.sg_windows(walks, R)
    noise = rng.integers(0, V, size=(len(ins), 2 * R, K))
    loss, gi, go, rec, prec = sgns_ref.sgns_forward_backward(w_in0, w_out0, ins, tgt, noise)
    w_in, w_out = _dev(w_in0), _dev(w_out0)
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, walks=_dev(walks), context_radius=R,
                          noise=_dev(noise))
    t = loss_terms(acc, tgt.size, K)
    assert float(t['loss']) == pytest.approx(loss['loss'], rel=1e-5)
    scale = float(np.abs(gi).max())
    np.testing.assert_allclose(g_in.cpu().numpy(), gi, rtol=1e-4, atol=1e-6 * scale)
    np.testing.assert_allclose(g_out.cpu().numpy(), go, rtol=1e-4, atol=1e-6 * scale)
    # the atomic path agrees with the sorted one
    g_in2, g_out2 = torch.zeros_like(w_in), torch.zeros_like(w_out)
    sgns_accumulate(w_in, w_out, g_in2, g_out2, K, walks=_dev(walks), context_radius=R,
                    noise=_dev(noise), scatter='atomic')
    torch.testing.assert_close(g_out2, g_out, rtol=1e-4, atol=1e-6 * scale)
    torch.testing.assert_close(g_in2, g_in, rtol=1e-4, atol=1e-6 * scale)
    # the sorted path is reproducible run to run (stable sort, fixed per-row summation order)
    if not hub:
        g_in3, g_out3 = torch.zeros_like(w_in), torch.zeros_like(w_out)
        sgns_accumulate(w_in, w_out, g_in3, g_out3, K, walks=_dev(walks), context_radius=R,
                        noise=_dev(noise))
        assert torch.equal(g_out3, g_out)


def test_device_noise_matches_philox_oracle(hip_device):
    f = golden('sgns_d128_k5.npz')
    w_in, w_out = _tables(f)
    K, R, V = int(f['K']), int(f['R']), int(f['V'])
    g1, o1 = torch.zeros_like(w_in), torch.zeros_like(w_out)
    acc1 = sgns_accumulate(w_in, w_out, g1, o1, K, walks=_dev(f['walks'], torch.int32),
                           context_radius=R, noise=None, seed=1234, noise_offset=5000)
    nz = ph.device_noise(1234, 5000, f['targets'].shape[0], 2 * R, K, V)
    g2, o2 = torch.zeros_like(w_in), torch.zeros_like(w_out)
    acc2 = sgns_accumulate(w_in, w_out, g2, o2, K, walks=_dev(f['walks'], torch.int32),
                           context_radius=R, noise=_dev(nz, torch.int64))
    torch.testing.assert_close(acc1, acc2, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(g1, g2, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(o1, o2, rtol=1e-6, atol=1e-9)


def test_bad_index_is_reported_not_faulting(hip_device):
    f = golden('sgns_karate_d2_k1.npz')
    w_in, w_out = _tables(f)
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    noise = torch.as_tensor(f['noise'][0]).clone()
    noise[3, 1, 0] = 10_000
    status = torch.zeros(1, dtype=torch.int32, device='cuda')
    sgns_accumulate(w_in, w_out, g_in, g_out, 1, inputs=_dev(f['inputs'], torch.int64),
                    targets=_dev(f['targets'], torch.int64), noise=_dev(noise, torch.int64),
                    status=status)
    with pytest.raises(IndexError):
        _native.check_status(status, 'sgns')


def test_skipgram_forward_backward_vs_oracle(hip_device):
    f = golden('sgns_d128_k5.npz')
    torch.manual_seed(0)
    m = SkipGram(int(f['V']), int(f['d'])).cuda()
    with torch.no_grad():
        m._input_embedding.weight.copy_(torch.as_tensor(f['w_in0']))
        m._output_embedding.weight.copy_(torch.as_tensor(f['w_out0']))
    ins = _dev(f['inputs'], torch.int64)
    tgt = _dev(f['targets'], torch.int64)
    logits = m(ins, tgt, proba=False)
    win = torch.tensor(f['w_in0'], requires_grad=True)
    wout = torch.tensor(f['w_out0'], requires_grad=True)
    ref = sgns_ref.skipgram_logits(win, wout, torch.as_tensor(f['inputs']),
                                   torch.as_tensor(f['targets']))
    np.testing.assert_allclose(logits.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5,
                               atol=1e-7)
    wt = torch.as_tensor(np.random.default_rng(0).standard_normal(ref.shape).astype(np.float32))
    (logits * wt.cuda()).sum().backward()
    (ref * wt).sum().backward()
    np.testing.assert_allclose(m._input_embedding.weight.grad.cpu().numpy(), win.grad.numpy(),
                               rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(m._output_embedding.weight.grad.cpu().numpy(), wout.grad.numpy(),
                               rtol=1e-4, atol=1e-7)
    probs = m(ins, tgt, proba=True)
    torch.testing.assert_close(probs, torch.sigmoid(logits))


def test_autograd_path_equals_manual_path(hip_device):
    f = golden('sgns_d128_k5.npz')
    w_in = torch.nn.Parameter(_dev(f['w_in0'], torch.float32))
    w_out = torch.nn.Parameter(_dev(f['w_out0'], torch.float32))
    noise = _dev(f['noise'][0], torch.int64)
    outs = SGNSLoss.apply(w_in, w_out, _dev(f['inputs'], torch.int64).reshape(-1),
                          _dev(f['targets'], torch.int64), noise, 2, int(f['K']), 0, 0)
    (outs[0] * 3.0).backward()
    np.testing.assert_allclose(w_in.grad.cpu().numpy(), 3.0 * f['g_in'], rtol=1e-5, atol=1e-8)
    np.testing.assert_allclose(w_out.grad.cpu().numpy(), 3.0 * f['g_out'], rtol=1e-5, atol=1e-8)


# ---- CBOW (pooled inputs) and nn.Embedding(max_norm) renormalisation -------
def _max_norm(f):
    return None if np.isnan(float(f['max_norm'])) else float(f['max_norm'])


@pytest.mark.parametrize('name', POOLED_FIXTURES)
def test_cbow_and_max_norm_step_vs_reference(name, hip_device):
    """Renormalise the looked-up rows like the reference's two forwards, then one fused step
    (dw_sgns_pooled_pairs for CBOW) — loss, metrics, renormalised tables and gradients."""
    from shallow_encoders.word2vec.sgns import renorm_
    f = golden(name)
    mn = _max_norm(f)
    w_in, w_out = _dev(f['w_in0']), _dev(f['w_out0'])
    inputs, targets = _dev(f['inputs'], torch.long), _dev(f['targets'], torch.long)
    noise = _dev(f['noise'][0], torch.long)
    B, C = targets.shape
    K = int(f['K'])
    if mn is not None:
        renorm_(w_in, inputs, mn)
        renorm_(w_out, targets, mn)
        renorm_(w_out, noise, mn)
    # norms: wave-order float sum vs torch's; the renormalised rows agree to a few ulp
    np.testing.assert_allclose(w_in.cpu().numpy(), f['w_in0r'], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(w_out.cpu().numpy(), f['w_out0r'], rtol=1e-6, atol=1e-7)
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, inputs=inputs, targets=targets,
                          noise=noise)
    t = loss_terms(acc, B * C, K)
    np.testing.assert_allclose([float(t['loss']), float(t['positive-loss']),
                                float(t['negative-loss'])], f['losses'][0], rtol=1e-5)
    assert float(t['recall']) == pytest.approx(float(f['recall'][0]), abs=1e-6)
    assert float(t['precision']) == pytest.approx(float(f['precision'][0]), abs=1e-6)
    assert_grad_close(g_in.cpu().numpy(), f['g_in'])
    assert_grad_close(g_out.cpu().numpy(), f['g_out'])


@pytest.mark.parametrize('name', POOLED_FIXTURES)
def test_cbow_and_max_norm_adam_steps_vs_reference(name, hip_device):
    """Renormalise + fused step + HIP dense Adam for every recorded batch: parameters after the
    first step and the loss of every step against the reference's own training."""
    from shallow_encoders.word2vec.sgns import renorm_
    from shallow_encoders.word2vec.sharding import ShardedTables
    f = golden(name)
    mn = _max_norm(f)
    V, d, K, lr = int(f['V']), int(f['d']), int(f['K']), float(f['lr'])
    t = ShardedTables(V, d, hip_device, lr=lr, init_seed=None)
    t.load_(torch.as_tensor(f['w_in0']), torch.as_tensor(f['w_out0']))
    inputs, targets = _dev(f['inputs'], torch.long), _dev(f['targets'], torch.long)
    B, C = targets.shape
    for step in range(f['noise'].shape[0]):
        noise = _dev(f['noise'][step], torch.long)
        if mn is not None:
            renorm_(t.w_in, inputs, mn)
            renorm_(t.w_out, targets, mn)
            renorm_(t.w_out, noise, mn)
        acc = sgns_accumulate(t.w_in, t.w_out, t.g_in, t.g_out, K, inputs=inputs,
                              targets=targets, noise=noise)
        assert float(loss_terms(acc, B * C, K)['loss']) == pytest.approx(
            float(f['losses'][step][0]), rel=1e-4)
        t.step()
        if step == 0:   # tiny tables: allow 2 sign-flipped near-zero-gradient entries
            frac = max(1e-3, 2.0 / t.w_in.numel())
            assert_params_close(t.w_in.cpu().numpy(), f['w_in1'], lr, max_frac=frac,
                                max_abs=2.05 * lr)
            assert_params_close(t.w_out.cpu().numpy(), f['w_out1'], lr, max_frac=frac,
                                max_abs=2.05 * lr)


def test_cbow_forward_backward_vs_oracle(hip_device):
    """CBOW.forward (dw_pooled_logits) and its backward against model.py:102-107 on the CPU."""
    from shallow_encoders.word2vec.model import CBOW
    f = golden('sgns_cbow_d16_k3.npz')
    V, d = int(f['V']), int(f['d'])
    model = CBOW(V, d).to(hip_device)
    with torch.no_grad():
        model.input_weight.copy_(torch.as_tensor(f['w_in0']))
        model.output_weight.copy_(torch.as_tensor(f['w_out0']))
    inputs = torch.as_tensor(f['inputs'])
    outputs = torch.as_tensor(f['noise'][0]).reshape(inputs.shape[0], -1)
    logits = model(inputs, outputs, proba=False)
    (logits * torch.linspace(-1, 1, logits.numel(), device=hip_device).view_as(logits)).sum() \
        .backward()
    win = torch.tensor(f['w_in0'], requires_grad=True)
    wout = torch.tensor(f['w_out0'], requires_grad=True)
    ref = sgns_ref.pooled_logits(win, wout, inputs, outputs)
    (ref * torch.linspace(-1, 1, ref.numel()).view_as(ref)).sum().backward()
    np.testing.assert_allclose(logits.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5,
                               atol=1e-7)
    np.testing.assert_allclose(model.input_weight.grad.cpu().numpy(), win.grad.numpy(),
                               rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(model.output_weight.grad.cpu().numpy(), wout.grad.numpy(),
                               rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(model(inputs, outputs).detach().cpu().numpy(),
                               torch.sigmoid(ref).detach().numpy(), rtol=1e-5, atol=1e-7)


def test_device_noise_fill_matches_in_kernel_draws(hip_device):
    """dw_sgns_noise writes exactly the negatives the fused kernel draws for noise=None."""
    from shallow_encoders.word2vec.sgns import device_noise
    f = golden('sgns_d128_k5.npz')
    w_in, w_out = _dev(f['w_in0']), _dev(f['w_out0'])
    inputs, targets = _dev(f['inputs'], torch.long), _dev(f['targets'], torch.long)
    B, C = targets.shape
    K, V = int(f['K']), int(f['V'])
    outs = []
    for noise in (None, device_noise(B, C, K, V, 17, 1000, hip_device)):
        g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
        acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, inputs=inputs, targets=targets,
                              noise=noise, seed=17, noise_offset=1000, scatter='atomic')
        outs.append((acc.cpu().numpy(), g_in.cpu().numpy(), g_out.cpu().numpy()))
    np.testing.assert_allclose(outs[0][0], outs[1][0], rtol=1e-6)
    assert_grad_close(outs[1][1], outs[0][1])
    assert_grad_close(outs[1][2], outs[0][2])
    ref = ph.device_noise(17, 1000, B, C, K, V)
    np.testing.assert_array_equal(device_noise(B, C, K, V, 17, 1000, hip_device).cpu().numpy(),
                                  ref.reshape(B, C, K))


@pytest.mark.parametrize('d,nw', [(64, 256), (100, 256), (128, 256), (128, 255)])
def test_fused_out_table_adam_equals_unfused(hip_device, d, nw):
    """dw_sgns_walks_phase2_adam (the output table's Adam fused into the records gather) gives
    the tables that phase 2 + dw_adam_dense give, over several steps; g_out and the row flags
    are left zeroed. Float atomics (g_in, chunk-boundary rows) make two runs of either path
    differ in the last bits, which Adam amplifies only where a gradient is ~0: the tables are
    compared with the Adam-aware tolerance of assert_params_close."""
    from shallow_encoders.graph.random_walk_generator import DeepWalk
    from shallow_encoders.graph.rmat import rmat_graph
    from shallow_encoders.word2vec.sharding import ShardedTables
    csr = rmat_graph(12, 40_000, 0, device=hip_device)
    walker = DeepWalk(csr, 40, rng='philox', seed=3, device=hip_device)
    V, R, K = csr.vocab_size, 3, 4   # nw = 255: records % 8 != 0 (a partial last group)
    fused = ShardedTables(V, d, hip_device, lr=0.02, init_seed=5)
    plain = ShardedTables(V, d, hip_device, lr=0.02, init_seed=5)
    for step in range(3):
        starts = torch.randint(1, V, (nw,), generator=torch.Generator().manual_seed(step),
                               dtype=torch.int32).to(hip_device)
        walks = walker.walk_batch(starts, walk_id0=step * nw)
        for t, fuse in ((fused, True), (plain, False)):
            kw = dict(walks=walks, context_radius=R, seed=7, noise_offset=step * nw * 34)
            sgns_accumulate(t.w_in, t.w_out, t.g_in, t.g_out, K, phase=1, **kw)
            t.exchange_in()
            spec = t.out_adam_spec() if fuse else None
            assert (spec is not None) == fuse
            sgns_accumulate(t.w_in, t.w_out, t.g_in, t.g_out, K, phase=2, out_adam=spec, **kw)
            t.exchange_out(fused_out=fuse)
            t.sync()
    torch.cuda.synchronize()
    assert float(fused.grads.abs().max()) == 0.0
    assert int(fused._row_flags.max()) == 0
    for a, b in ((fused.w_in, plain.w_in), (fused.w_out, plain.w_out)):
        assert_params_close(a.cpu().numpy(), b.cpu().numpy(), 0.02, max_frac=5e-3,
                            max_abs=2.05 * 0.02 * 3)
        assert_no_row_drift(a.cpu().numpy(), b.cpu().numpy())
    np.testing.assert_allclose(fused.m.cpu().numpy(), plain.m.cpu().numpy(), rtol=1e-3,
                               atol=1e-6)
