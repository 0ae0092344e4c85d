"""Dense Adam on gfx950 — the optimizer the reference configs name (``torch.optim.Adam``,
configs/sge_sg_*.yaml; instantiated at config_parser/core.py:43-53).

Same hyper-parameters, state names (``step``, ``exp_avg``, ``exp_avg_sq``) and update as
torch's single-tensor Adam (torch/optim/adam.py, amsgrad=False); the scalars are computed on
the host in float64 exactly as torch computes them, the tensor update runs in one streaming
kernel per parameter (dw_adam_dense) that can also zero the gradient in the same pass
(``zero_grad_in_step=True``: saves the separate zero_grad pass over V x d).

Fused form (``fuse_into_sgns=True``, the default): when this optimizer holds exactly a model's
two embedding tables, Word2VecTrainer's walk-batch step applies the update itself, inside the
SGNS kernels (the output table's Adam in the records gather, the input table's on a side
stream overlapping it; see Word2VecTrainer._fused_walk_step). It claims the step with
``begin_fused_step``, and the ``step()`` that follows skips those parameters once.
"""
from typing import Dict, Iterable, List, Tuple

import torch
from torch.optim import Optimizer

from shallow_encoders import _native


class Adam(Optimizer):
    """Adam with the math of ``torch.optim.Adam`` (dense; every row moves every step)."""

    def __init__(self, params: Iterable, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, amsgrad: bool = False, *,
                 zero_grad_in_step: bool = True, fuse_into_sgns: bool = True, **unsupported):
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
        self.fuse_into_sgns = fuse_into_sgns
        self._fused_done = set()   # ids of parameters whose update this step already applied
        self._alt: Dict[int, torch.Tensor] = {}   # second buffer of double-buffered parameters
        # ids of parameters whose .grad is known to be all zero (a fresh buffer, or one a
        # zeroing step consumed): the fused step needs it — its interior rows never read g
        self._grads_clean = set()

    # ---- fused form ---------------------------------------------------------------------------
    def can_fuse(self, params: List[torch.Tensor]) -> bool:
        """True when this optimizer's update of exactly ``params`` (one group, HIP fp32
        contiguous tensors, gradients zeroed by the step) may run inside the SGNS step."""
        if not (self.fuse_into_sgns and self.zero_grad_in_step) or len(self.param_groups) != 1:
            return False
        mine = self.param_groups[0]['params']
        if len(mine) != len(params) or {id(p) for p in mine} != {id(p) for p in params}:
            return False
        return all(p.device.type == 'cuda' and p.dtype == torch.float32 and p.is_contiguous()
                   and p.grad is not None and p.grad.is_contiguous()
                   and id(p) in self._grads_clean for p in params)

    def mark_grads(self, params: List[torch.Tensor], clean: bool) -> None:
        """Record that the gradients of ``params`` are all zero (``clean``: a new zero buffer)
        or may not be (something accumulated into them outside a fused step)."""
        for p in params:
            (self._grads_clean.add if clean else self._grads_clean.discard)(id(p))

    def begin_fused_step(self, params: List[torch.Tensor]) -> List[Tuple[dict, tuple]]:
        """Count one step for each of ``params`` (state created on first use) and return
        ``(state, dw_adam_dense scalars)`` per parameter; the next ``step()`` skips them."""
        out = []
        group = self.param_groups[0]
        for p in params:
            state = self._state_of(p)
            state['step'] += 1
            out.append((state, self._scalars(group, float(state['step'].item()))))
            self._fused_done.add(id(p))
            self._grads_clean.add(id(p))     # the fused step leaves the gradient zero
        return out

    def alt_buffer(self, p: torch.Tensor) -> torch.Tensor:
        """The second buffer of a double-buffered parameter (allocated once)."""
        b = self._alt.get(id(p))
        if b is None or b.shape != p.shape or b.device != p.device:
            b = torch.empty_like(p)
            self._alt[id(p)] = b
        return b

    def swap_alt(self, p: torch.Tensor) -> None:
        """``p`` takes the second buffer's storage (just written by an out-of-place update);
        its old storage becomes the second buffer."""
        b = self._alt[id(p)]
        self._alt[id(p)] = p.data
        p.data = b

    def _state_of(self, p: torch.Tensor) -> dict:
        state = self.state[p]
        if len(state) == 0:
            state['step'] = torch.tensor(0.0, dtype=torch.float32)
            state['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
            state['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return state

    @staticmethod
    def _scalars(group: dict, step: float) -> tuple:
        """dw_adam_dense's scalars, float64 on the host as torch derives them."""
        beta1, beta2 = group['betas']
        bias_correction1 = 1 - beta1 ** step
        bias_correction2 = 1 - beta2 ** step
        return (1 - beta1, beta2, 1 - beta2, bias_correction2 ** 0.5,
                -(group['lr'] / bias_correction1), group['eps'], group['weight_decay'])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        done, self._fused_done = self._fused_done, set()
        for group in self.param_groups:
            for p in group['params']:
                if p.grad is None or id(p) in done:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError('HIP Adam does not support sparse gradients')
                if p.dtype != torch.float32 or p.device.type != 'cuda':
                    raise TypeError('HIP Adam needs float32 parameters on a HIP device')
                state = self._state_of(p)
                state['step'] += 1
                scalars = self._scalars(group, float(state['step'].item()))
                g = p.grad
                if not g.is_contiguous():
                    g = g.contiguous()
                    p.grad = g
                with torch.cuda.device(p.device):
                    _native.call('dw_adam_dense', _native.ptr(p), _native.ptr(g),
                                 _native.ptr(state['exp_avg']), _native.ptr(state['exp_avg_sq']),
                                 p.numel(), *scalars, 1 if self.zero_grad_in_step else 0,
                                 _native.stream(p.device))
                self.mark_grads([p], self.zero_grad_in_step)
        return loss

    def zero_grad(self, set_to_none: bool = True) -> None:
        """With ``zero_grad_in_step`` the step already left every gradient zero: keep the
        buffers (no extra pass, no reallocation). Otherwise behave like torch."""
        if self.zero_grad_in_step:
            return
        super().zero_grad(set_to_none=set_to_none)
