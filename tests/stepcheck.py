"""One training step checked from the state the product held before it (test helper).

The reference step (oracle): the float64 closed-form gradient of the batch-mean loss
(oracle.sgns_ref.sgns_grads_closed_form_torch: loss.py:14-22 + the autograd gradient of
trainer.py:131-152) over the batch's windows (sg_windows_torch) and device negatives
(oracle.philox.device_noise_torch), then one torch.optim.Adam(foreach=False) step (the reference's
optimizer, config_parser/core.py:43-53) on the same (p, m, v), given that gradient rounded to
float32. The bars are the single-step ones of tests/test_gpu_c3_step.py, with
no fraction allowance:
  * gradient (first step only, read back as m / (1 - beta1)): rtol 1e-5, atol 2e-6 max|g|;
  * m: rtol 1e-5, atol (1 - beta1) g_atol; v: rtol 1e-4 plus its square term;
  * parameters: rtol 1e-5, atol 1e-6;
  * the update p1 - p0: rtol 1e-3, atol 1e-8 + (lr / bc1)(1 - beta1) g_atol / eps (the gradient's
    bar carried through Adam's 1 / (sqrt(v) + eps)).
"""
import numpy as np
import torch

from oracle import philox as ph
from oracle import sgns_ref

BETAS, EPS = (0.9, 0.999), 1e-8


def reference_grads(p_in, p_out, walks, R, K, seed, noise_offset):
    """(loss sums, g_in, g_out) float64 of the batch ``walks`` from tables (p_in, p_out)."""
    dev = p_in.device
    walks = torch.as_tensor(walks).to(dev)
    ins, tgt = sgns_ref.sg_windows_torch(walks, R)
    noise = ph.device_noise_torch(seed, noise_offset, ins.numel(), 2 * R, K, p_in.shape[0],
                                  device=dev)
    return sgns_ref.sgns_grads_closed_form_torch(p_in, p_out, ins, tgt, noise)


def _close(name, got, exp, rtol, atol):
    got, exp = torch.as_tensor(got).double(), torch.as_tensor(exp).double()
    err = (got - exp).abs()
    lim = atol + rtol * exp.abs()
    n_bad = int((err > lim).sum())
    worst = float((err / lim).max()) if err.numel() else 0.0
    assert n_bad == 0, f'{name}: {n_bad} of {got.numel()} entries outside rtol {rtol} / ' \
                       f'atol {atol:.3e} (worst err/limit {worst:.2f})'
    return worst


def check_adam_step(tag, g, pre, post, step, lr, betas=BETAS, eps=EPS):
    """pre / post: (p, m, v) before and after Adam step ``step`` (1-based) with gradient g
    (float64). Returns {quantity: worst err/limit}."""
    p0, m0, v0 = (torch.as_tensor(x).float().cpu() for x in pre)
    p1, m1, v1 = (torch.as_tensor(x).float().cpu() for x in post)
    g = torch.as_tensor(g).double().cpu()
    b1, b2 = betas
    pr = p0.clone().requires_grad_()
    opt = torch.optim.Adam([pr], lr=lr, betas=betas, eps=eps, foreach=False)
    if step > 1:
        opt.state[pr] = {'step': torch.tensor(float(step - 1)), 'exp_avg': m0.clone(),
                         'exp_avg_sq': v0.clone()}
    pr.grad = g.float()
    opt.step()
    st = opt.state[pr]
    gmax = float(g.abs().max()) if g.numel() else 0.0
    g_atol = 2e-6 * gmax
    res = {}
    if step == 1:
        res['g'] = _close(f'{tag} g', m1.double() / float(np.float32(1 - b1)), g, 1e-5, g_atol)
    res['m'] = _close(f'{tag} m', m1, st['exp_avg'], 1e-5, (1 - b1) * g_atol)
    res['v'] = _close(f'{tag} v', v1, st['exp_avg_sq'], 1e-4, (1 - b2) * (2 * gmax + g_atol) * g_atol)
    res['p'] = _close(f'{tag} p', p1, pr.detach(), 1e-5, 1e-6)
    dp_atol = 1e-8 + lr / (1 - b1 ** step) * (1 - b1) * g_atol / eps
    res['dp'] = _close(f'{tag} dp', p1.double() - p0.double(), pr.detach().double() - p0.double(),
                       1e-3, dp_atol)
    return res


def check_trajectory(tag, init, snaps, walks_all, R, K, seed, lr, centres_per_step):
    """Every step of a run: init = (w_in, w_out) before step 1; snaps[s] = (w_in, w_out, m_in,
    v_in, m_out, v_out) after step s + 1 (full tables); walks_all[s] the step's global batch,
    its negatives at noise offset s * centres_per_step. Each step from the snapshot before it."""
    w_in, w_out = (torch.as_tensor(np.asarray(x)) for x in init)
    z = torch.zeros_like(w_in)
    pre = (w_in, w_out, z, z, z.clone(), z.clone())
    worst = {}
    for s, post in enumerate(snaps):
        post = tuple(torch.as_tensor(np.asarray(x)) for x in post)
        dev = 'cuda' if torch.cuda.is_available() else 'cpu'
        _, gi, go = reference_grads(pre[0].to(dev), pre[1].to(dev), walks_all[s], R, K, seed,
                                    s * centres_per_step)
        for name, g, i in (('in', gi, (0, 2, 3)), ('out', go, (1, 4, 5))):
            r = check_adam_step(f'{tag} step {s + 1} {name}', g, [pre[k] for k in i],
                                [post[k] for k in i], s + 1, lr)
            for q, w in r.items():
                worst[f'{q}_{name}'] = max(worst.get(f'{q}_{name}', 0.0), w)
        pre = post
    return worst
