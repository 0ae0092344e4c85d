"""Embedding tables sharded by node-id range across the GPUs of one node.

The reference trains on one device (``devices: '1'`` in every config). Data-parallel SGNS
with dense Adam semantics is laid out here ZeRO-1 style, one process per GPU:

  params  float32 [2, V_pad, d]   both tables (in, out) in ONE flat buffer, replicated
  grads   float32 [2, V_pad, d]   local dense gradients (the fused SGNS kernel adds into them)
  m, v    float32 [2*V_pad*d / world]  Adam state for THIS rank's contiguous slice only

Per optimizer step (all collectives over RCCL = torch.distributed 'nccl' on ROCm, xGMI):
  1. reduce-scatter(sum) of the flat gradient: rank r receives the global gradient of its
     slice — a contiguous node-id range of the stacked [in; out] tables;
  2. dense Adam on that slice only (dw_adam_dense): 1/world of the optimizer's HBM traffic;
  3. all-gather of the updated parameter slices back into every rank's replica.
Every rank scales its local gradient by 1/M_global (the mean over the GLOBAL batch), so the
result equals single-device training on the concatenated batch (DDP semantics).
Walk generation needs no communication (walks are keyed by global walk id).

The Adam update is injectable (``adam_impl``) so the exchange logic can be tested with gloo
on CPU; the default is the HIP kernel and refuses host tensors.
"""
import math
from typing import Callable, Optional

import torch
import torch.distributed as dist

from shallow_encoders import _native


def hip_adam(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
             lr: float, betas, eps: float, weight_decay: float, zero_grad: bool) -> None:
    """One dense Adam step on flat fp32 buffers with torch.optim.Adam's scalar math."""
    beta1, beta2 = betas
    bias_correction1 = 1 - beta1 ** step
    bias_correction2 = 1 - beta2 ** step
    step_size = lr / bias_correction1
    with torch.cuda.device(p.device):
        _native.call('dw_adam_dense', _native.ptr(p), _native.ptr(g), _native.ptr(m),
                     _native.ptr(v), p.numel(), 1 - beta1, beta2, 1 - beta2,
                     bias_correction2 ** 0.5, -step_size, eps, weight_decay,
                     1 if zero_grad else 0, _native.stream(p.device))


class ShardedTables:
    """In/out embedding tables + dense gradients + node-range-sharded Adam state."""

    def __init__(self, vocab_size: int, dim: int, device, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 group=None, init_seed: Optional[int] = 0,
                 adam_impl: Optional[Callable] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.V, self.d = int(vocab_size), int(dim)
        self.V_pad = int(math.ceil(self.V / self.world)) * self.world
        self.device = torch.device(device)
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.adam_impl = adam_impl or hip_adam
        self.step_count = 0
        self.params = torch.zeros((2, self.V_pad, self.d), dtype=torch.float32, device=self.device)
        self.grads = torch.zeros_like(self.params)
        n = self.params.numel()
        self.shard_elems = n // self.world
        self.m = torch.zeros(self.shard_elems, dtype=torch.float32, device=self.device)
        self.v = torch.zeros_like(self.m)
        self.grad_shard = torch.empty_like(self.m) if self.world > 1 else None
        if init_seed is not None:
            self.xavier_(init_seed)

    # ---- views -------------------------------------------------------------------------------
    @property
    def w_in(self) -> torch.Tensor:
        return self.params[0, :self.V]

    @property
    def w_out(self) -> torch.Tensor:
        return self.params[1, :self.V]

    @property
    def g_in(self) -> torch.Tensor:
        return self.grads[0, :self.V]

    @property
    def g_out(self) -> torch.Tensor:
        return self.grads[1, :self.V]

    def shard_range(self):
        """[start, end) of this rank's slice in the flat [2*V_pad*d] parameter buffer."""
        return self.rank * self.shard_elems, (self.rank + 1) * self.shard_elems

    def xavier_(self, seed: int) -> None:
        """W2VBase init (model.py:26-27): U(-a, a), a = sqrt(6/(V+d)); identical on all ranks."""
        g = torch.Generator(device='cpu').manual_seed(int(seed))
        a = math.sqrt(6.0 / (self.V + self.d))
        for t in range(2):
            w = torch.rand((self.V, self.d), generator=g) * (2 * a) - a
            self.params[t, :self.V].copy_(w)

    def load_(self, w_in: torch.Tensor, w_out: torch.Tensor) -> None:
        self.params[0, :self.V].copy_(w_in)
        self.params[1, :self.V].copy_(w_out)

    # ---- optimizer step ---------------------------------------------------------------------------
    def step(self) -> None:
        """Exchange gradients, update this rank's slice, gather parameters; grads end zeroed."""
        self.step_count += 1
        flat_p = self.params.view(-1)
        flat_g = self.grads.view(-1)
        if self.world == 1:
            self.adam_impl(flat_p, flat_g, self.m, self.v, self.step_count, self.lr, self.betas,
                           self.eps, self.weight_decay, True)
            return
        dist.reduce_scatter_tensor(self.grad_shard, flat_g, op=dist.ReduceOp.SUM,
                                   group=self.group)
        flat_g.zero_()
        a, b = self.shard_range()
        p_shard = flat_p[a:b]
        self.adam_impl(p_shard, self.grad_shard, self.m, self.v, self.step_count, self.lr,
                       self.betas, self.eps, self.weight_decay, False)
        backend = dist.get_backend(self.group)
        src = p_shard if backend == 'nccl' else p_shard.clone()  # RCCL all-gather is in-place safe
        dist.all_gather_into_tensor(flat_p, src, group=self.group)
