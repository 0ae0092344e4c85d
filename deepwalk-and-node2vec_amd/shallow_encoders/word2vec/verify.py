"""A training step checked by the run itself on a sample of rows (bench.py's self-check of the
N > 1 line, which no single-GPU box can rehearse at scale).

The expected step is restated here in float64 torch on the device, from the full tables as they
stood before the step: the batch's skip-gram windows (torch_dataset.py:293-322), the device
negatives the SGNS pass draws (dw_sgns_noise: the same Philox keys), the closed-form gradient of
the batch-mean NegativeSamplingLoss (loss.py:14-22, including its clamp(sigmoid, 1e-6) zero
gradient) that autograd gives the reference's training_step (trainer.py:131-152), restricted to
the sampled rows, then one torch.optim.Adam(foreach=False) step (config_parser/core.py:43-53) of
those rows. The bars are the single-step ones of the parity tests (tests/stepcheck.py):
gradient rtol 1e-5 / atol 2e-6 max|g| (seen through m), parameters rtol 1e-5 / atol 1e-6, the
update p1 - p0 rtol 1e-3 with the gradient's bar carried through Adam's normalisation.
"""
from typing import Dict, Optional, Tuple

import torch

from shallow_encoders.word2vec.sgns import device_noise


def windows(walks: torch.Tensor, radius: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(centres [B'], contexts [B', 2R]) int64 in the collate's order (left then right)."""
    n, L = walks.shape
    centres = torch.arange(radius, L - radius, device=walks.device)
    off = torch.cat([torch.arange(-radius, 0), torch.arange(1, radius + 1)]).to(walks.device)
    w = walks.long()
    return w[:, centres].reshape(-1), w[:, centres[:, None] + off[None, :]].reshape(-1, 2 * radius)


def sampled_grads(w_in: torch.Tensor, w_out: torch.Tensor, walks: torch.Tensor, R: int, K: int,
                  seed: int, noise_offset: int, rows_in: torch.Tensor, rows_out: torch.Tensor,
                  chunk: int = 4096) -> Tuple[torch.Tensor, torch.Tensor]:
    """float64 gradients of the batch-mean loss for the rows ``rows_in`` of the in table and
    ``rows_out`` of the out table (distinct ids), from full (V, d) tables."""
    dev = w_in.device
    V, d = w_in.shape
    ins, tgt = windows(walks.to(dev), R)
    B, C = tgt.shape
    noise = device_noise(B, C, K, V, seed, noise_offset, dev)
    M = float(B * C)
    pos_in = torch.full((V,), -1, dtype=torch.int64, device=dev)
    pos_in[rows_in] = torch.arange(rows_in.numel(), device=dev)
    pos_out = torch.full((V,), -1, dtype=torch.int64, device=dev)
    pos_out[rows_out] = torch.arange(rows_out.numel(), device=dev)
    g_in = torch.zeros((rows_in.numel(), d), dtype=torch.float64, device=dev)
    g_out = torch.zeros((rows_out.numel(), d), dtype=torch.float64, device=dev)
    for a in range(0, B, chunk):
        b = min(B, a + chunk)
        ii, tt, nn = ins[a:b], tgt[a:b], noise[a:b]
        c = w_in[ii].double()
        o = w_out[tt].double()
        ng = w_out[nn].double()
        s = torch.einsum('bd,bjd->bj', c, o)
        t = torch.einsum('bd,bjkd->bjk', c, ng)
        sig_s, sig_t = torch.sigmoid(s), torch.sigmoid(t)
        ds = torch.where(sig_s >= 1e-6, sig_s - 1.0, torch.zeros_like(s)) / M
        dt = torch.where(torch.sigmoid(-t) >= 1e-6, sig_t, torch.zeros_like(t)) / M
        pi = pos_in[ii]
        m = pi >= 0
        if bool(m.any()):
            gc = torch.einsum('bj,bjd->bd', ds[m], o[m]) + torch.einsum('bjk,bjkd->bd', dt[m],
                                                                        ng[m])
            g_in.index_add_(0, pi[m], gc)
        pt = pos_out[tt]
        m = pt >= 0
        if bool(m.any()):
            g_out.index_add_(0, pt[m], (ds[..., None] * c[:, None, :])[m])
        pn = pos_out[nn]
        m = pn >= 0
        if bool(m.any()):
            g_out.index_add_(0, pn[m], (dt[..., None] * c[:, None, None, :])[m])
    return g_in, g_out


def _close(got: torch.Tensor, exp: torch.Tensor, rtol: float, atol: float) -> Tuple[int, float]:
    got, exp = got.double(), exp.double()
    err = (got - exp).abs()
    lim = atol + rtol * exp.abs()
    return int((err > lim).sum()), float((err / lim).max()) if err.numel() else 0.0


def check_rows(g: torch.Tensor, pre: Tuple[torch.Tensor, ...], post: Tuple[torch.Tensor, ...],
               step: int, lr: float, betas=(0.9, 0.999), eps: float = 1e-8,
               weight_decay: float = 0.0) -> Dict[str, Tuple[int, float]]:
    """{quantity: (entries outside the bar, worst err / limit)} of one Adam step of the sampled
    rows: pre / post = (p, m, v) before and after step ``step``; g their float64 gradient."""
    p0, m0, v0 = (x.float().cpu() for x in pre)
    p1, m1, v1 = (x.float().cpu() for x in post)
    g = g.double().cpu()
    pr = p0.clone().requires_grad_()
    opt = torch.optim.Adam([pr], lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                           foreach=False)
    if step > 1:
        opt.state[pr] = {'step': torch.tensor(float(step - 1)), 'exp_avg': m0.clone(),
                         'exp_avg_sq': v0.clone()}
    pr.grad = g.float()
    opt.step()
    st = opt.state[pr]
    b1, b2 = betas
    gmax = float(g.abs().max()) if g.numel() else 0.0
    g_atol = 2e-6 * gmax
    res = {'m': _close(m1, st['exp_avg'], 1e-5, (1 - b1) * g_atol + 1e-30),
           'v': _close(v1, st['exp_avg_sq'], 1e-4, (1 - b2) * (2 * gmax + g_atol) * g_atol + 1e-30),
           'p': _close(p1, pr.detach(), 1e-5, 1e-6)}
    dp_atol = 1e-8 + lr / (1 - b1 ** step) * (1 - b1) * g_atol / eps
    res['dp'] = _close(p1.double() - p0.double(), pr.detach().double() - p0.double(), 1e-3,
                       dp_atol)
    return res


def sample_rows(walks: torch.Tensor, R: int, K: int, V: int, seed: int, noise_offset: int,
                n: int, gen: Optional[torch.Generator] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Up to n distinct in rows (the batch's centres) and n out rows (its contexts and
    negatives), plus a few rows the batch does not touch (their g = 0 step), sorted."""
    dev = walks.device
    ins, tgt = windows(walks, R)
    B, C = tgt.shape
    noise = device_noise(B, C, K, V, seed, noise_offset, dev)
    g = gen or torch.Generator().manual_seed(0)

    def pick(ids: torch.Tensor) -> torch.Tensor:
        u = torch.unique(ids.reshape(-1)).cpu()
        sel = u[torch.randperm(u.numel(), generator=g)[:n]]
        extra = torch.randint(1, V, (max(1, n // 8),), generator=g)
        return torch.unique(torch.cat([sel, extra])).to(dev)
    return pick(ins), pick(torch.cat([tgt.reshape(-1), noise.reshape(-1)]))


def summarize(res: Dict[str, Dict[str, Tuple[int, float]]]) -> Dict[str, object]:
    """{'ok', 'bad', 'worst'} over every table and quantity."""
    bad = {f'{t}.{q}': r[0] for t, rr in res.items() for q, r in rr.items() if r[0]}
    worst = {f'{t}.{q}': round(r[1], 4) for t, rr in res.items() for q, r in rr.items()}
    return {'ok': not bad, 'bad': bad, 'worst_err_over_limit': worst}

