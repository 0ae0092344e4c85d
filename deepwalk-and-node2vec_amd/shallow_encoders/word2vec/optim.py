"""Dense Adam on gfx950 — the optimizer the reference configs name (``torch.optim.Adam``,
configs/sge_sg_*.yaml; instantiated at config_parser/core.py:43-53).

Same hyper-parameters, state names (``step``, ``exp_avg``, ``exp_avg_sq``) and update as
torch's single-tensor Adam (torch/optim/adam.py, amsgrad=False); the scalars are computed on
the host in float64 exactly as torch computes them, the tensor update runs in one streaming
kernel per parameter (dw_adam_dense) that can also zero the gradient in the same pass
(``zero_grad_in_step=True``: saves the separate zero_grad pass over V x d).
"""
from typing import Iterable, Tuple

import torch
from torch.optim import Optimizer

from shallow_encoders import _native


class Adam(Optimizer):
    """Adam with the math of ``torch.optim.Adam`` (dense; every row moves every step)."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, amsgrad: bool = False, *,
                 zero_grad_in_step: bool = True, **unsupported):
        if unsupported:
            bad = {k: v for k, v in unsupported.items() if v not in (None, False)}
            if bad:
                raise NotImplementedError(f'HIP Adam does not support {sorted(bad)}')
        if amsgrad:
            raise NotImplementedError('HIP Adam does not implement amsgrad')
        if not 0.0 <= lr:
            raise ValueError(f'Invalid learning rate: {lr}')
        if not 0.0 <= eps:
            raise ValueError(f'Invalid epsilon value: {eps}')
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f'Invalid beta parameters: {betas}')
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        amsgrad=False)
        super().__init__(params, defaults)
        self.zero_grad_in_step = zero_grad_in_step

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group['betas']
            lr, eps, wd = group['lr'], group['eps'], group['weight_decay']
            for p in group['params']:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError('HIP Adam does not support sparse gradients')
                if p.dtype != torch.float32 or p.device.type != 'cuda':
                    raise TypeError('HIP Adam needs float32 parameters on a HIP device')
                state = self.state[p]
                if len(state) == 0:
                    state['step'] = torch.tensor(0.0, dtype=torch.float32)
                    state['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                state['step'] += 1
                step = float(state['step'].item())
                bias_correction1 = 1 - beta1 ** step
                bias_correction2 = 1 - beta2 ** step
                step_size = lr / bias_correction1
                bias_correction2_sqrt = bias_correction2 ** 0.5
                g = p.grad
                if not g.is_contiguous():
                    g = g.contiguous()
                    p.grad = g
                with torch.cuda.device(p.device):
                    _native.call('dw_adam_dense', _native.ptr(p), _native.ptr(g),
                                 _native.ptr(state['exp_avg']), _native.ptr(state['exp_avg_sq']),
                                 p.numel(), 1 - beta1, beta2, 1 - beta2, bias_correction2_sqrt,
                                 -step_size, eps, wd, 1 if self.zero_grad_in_step else 0,
                                 _native.stream(p.device))
        return loss

    def zero_grad(self, set_to_none: bool = True) -> None:
        """With ``zero_grad_in_step`` the step already left every gradient zero: keep the
        buffers (no extra pass, no reallocation). Otherwise behave like torch."""
        if self.zero_grad_in_step:
            return
        super().zero_grad(set_to_none=set_to_none)
