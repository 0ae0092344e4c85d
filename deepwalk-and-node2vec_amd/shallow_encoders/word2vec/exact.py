"""Deterministic accumulation ("race detection").

The default SGNS step sums the centre-table gradient rows, and the output-table rows that
straddle two gather chunks, with float atomics: the order of the additions is the order the
waves happen to reach L2, so two runs of the same configuration give tables that differ in the
last bits — and Adam's normalised steps turn that noise on g ~ 0 entries into lr-sized moves
over a run. In the deterministic mode every gradient term t (the fp32 product the kernel
forms) enters an int64 accumulator as round(t * 2^frac) (dw_exact_register): integer addition
is associative, so each gradient entry is the same integer whatever the order of the atomics,
the chunking of the records, the graph replay or the number of ranks the terms are spread over,
and its conversion back to fp32 is the same float. The tables are then bit-identical run to
run, eager and graph-replayed, on one rank and on N (tests/test_gpu_exact.py).

frac = dw_exact_frac_bits(grad_scale) = 32 + ceil(-log2 grad_scale): the terms are
|coef| <= grad_scale times table entries, so the quantum 2^-frac sits 2^32 below the largest
possible coefficient (a term keeps ~24 significant bits while the entries are ~2^-8 or more of
it) and a term stays inside the conversion's 2^51 for entries below 2^19; a term past it sets
DW_S_FIXED_RANGE (OverflowError at the next status check).

Cost: two int64 atomics or adds per term instead of one float FMA, the accumulators (8 B per
table entry) and one conversion of the sums (on the one-GPU dense path fused into the in-table
Adam: DW_EXACT_ADAM); bench.py --deterministic measures it.
Covered: the records (sorted) output path of dw_sgns_walks_phase / dw_sgns_pairs (skip-gram),
the fused output-table Adam, the owner layout (the centre sums reduce-scattered as int64), and
the lazy Adam tables (OwnerLazyTables.enable_exact: the rows-major out step's k_out_rows and
the COEFIN centre pass sum as integers, the pipelined steps included; at N > 1 the touched in
rows' sums are all-reduced as int64 and converted on every rank alike).
Not covered (refused): the atomic output scatter, pooled (CBOW) inputs, the replicated N > 1
layout's row pieces.
"""
import os
from typing import Dict, List, Optional

import torch

from shallow_encoders import _native


def enabled() -> bool:
    """DW_DETERMINISTIC=1 selects the deterministic mode for the trainer and the tables."""
    return os.environ.get('DW_DETERMINISTIC', '0') == '1'


def frac_bits(grad_scale: float) -> int:
    """The fixed-point scale (bits below the binary point) for terms bounded by grad_scale."""
    return int(_native.load().dw_exact_frac_bits(float(grad_scale)))


class FixedAccumulator:
    """The int64 twin of a float gradient buffer, registered with the library: SGNS launches
    that accumulate into ``grad`` add their terms into ``acc`` and convert the exact sums into
    ``grad`` (``defer``: the centre sums stay in ``acc`` for the caller's cross-rank reduction,
    then ``convert``)."""

    def __init__(self, grad: torch.Tensor, grad_scale: float, defer: bool = False,
                 adam: bool = False):
        if grad.dtype != torch.float32 or not grad.is_contiguous():
            raise TypeError('the gradient buffer must be contiguous float32')
        self.grad = grad
        self.frac = frac_bits(grad_scale)
        self.defer = bool(defer)
        # DW_EXACT_ADAM: the dense Adam over this buffer reads (and clears) the sums itself
        self.adam = bool(adam)
        self.acc = torch.zeros(grad.shape, dtype=torch.int64, device=grad.device)
        self._grad_ptr = grad.data_ptr()
        self._ptr = None            # the registered grad pointer while this one is active
        self.activate()

    def activate(self) -> None:
        """(Re-)register this accumulator as the one the library adds ``grad``'s terms into.
        Its int64 sums are zero between steps (every conversion clears them), so a cached
        accumulator is taken up again without clearing."""
        if self._ptr is None:
            _native.call('dw_exact_register', _native.ptr(self.grad), _native.ptr(self.acc),
                         self.grad.numel(), self.frac,
                         (_native.DW_EXACT_DEFER if self.defer else 0)
                         | (_native.DW_EXACT_ADAM if self.adam else 0))
            self._ptr = self._grad_ptr

    @property
    def active(self) -> bool:
        return self._ptr is not None

    def matches(self, grad: torch.Tensor, grad_scale: float) -> bool:
        return grad.data_ptr() == self._grad_ptr and self.frac == frac_bits(grad_scale)

    def convert(self, acc: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
                accumulate: bool = False) -> None:
        """out (default grad) = [out +] fl(acc * 2^-frac); acc (default self.acc) zeroed."""
        acc = self.acc if acc is None else acc
        out = self.grad if out is None else out
        if acc.numel() != out.numel():
            raise ValueError('accumulator and output sizes differ')
        with torch.cuda.device(out.device):
            _native.call('dw_fixed_to_float', _native.ptr(acc), _native.ptr(out), out.numel(),
                         self.frac, 1 if accumulate else 0, _native.stream(out.device))

    def release(self) -> None:
        """Unregister (only while active: another accumulator may hold the buffer since)."""
        if self._ptr is not None:
            _native.load().dw_exact_unregister(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.release()
        except Exception:   # interpreter shutdown
            pass


class Registry:
    """Accumulators per gradient buffer. A buffer's accumulator depends on the batch shape
    (grad_scale sets frac), and an epoch's short last batch changes it for one step and back:
    the accumulators are kept per (buffer, frac) for the registry's lifetime (at most
    ``MAX_PER_KEY`` per buffer; the least recently used inactive one is dropped past that) and
    re-registered, not reallocated, when the shape changes back. A captured graph keeps its
    own references (``live``), so its accumulators stay allocated whatever the registry does."""

    MAX_PER_KEY = 4

    def __init__(self):
        self._acc: Dict[int, FixedAccumulator] = {}                  # the active one per key
        self._cache: Dict[int, List[FixedAccumulator]] = {}          # per key, most recent last

    def ensure(self, key: int, grad: torch.Tensor, grad_scale: float,
               defer: bool = False, adam: bool = False) -> FixedAccumulator:
        def same(c):
            return c.matches(grad, grad_scale) and c.defer == defer and c.adam == adam
        a = self._acc.get(key)
        if a is not None and a.active and same(a):
            return a
        if a is not None:
            a.release()
        cache = self._cache.setdefault(key, [])
        hit = next((c for c in cache if same(c)), None)
        if hit is not None:
            cache.remove(hit)
            hit.activate()
        else:
            hit = FixedAccumulator(grad, grad_scale, defer, adam)
            while len(cache) >= self.MAX_PER_KEY:
                cache.pop(0)
        cache.append(hit)
        self._acc[key] = hit
        return hit

    def get(self, key: int) -> Optional[FixedAccumulator]:
        return self._acc.get(key)

    def live(self) -> List[FixedAccumulator]:
        """The active accumulators (what a graph captured now adds into)."""
        return [a for a in self._acc.values() if a.active]

    def release(self) -> None:
        for a in self._acc.values():
            a.release()
        self._acc = {}
        self._cache = {}
