"""Embedding tables sharded by node-id range across the GPUs of one node.

The reference trains on one device (``devices: '1'`` in every config). Here data-parallel SGNS
with dense Adam semantics is laid out ZeRO-1 style, one process per GPU. Every rank scales its
local gradient by 1/M_global (the mean over the GLOBAL batch), so the result equals
single-device training on the concatenated batch (DDP semantics). Walk generation needs no
communication, because walks are keyed by the global walk id.

Layout (P out-table pieces; V_pad = V rounded up to a multiple of world * P; S = V_pad / world):

  params  float32 [2 or 3, V_pad, d]   slot 1 = out table; slot 0 = in table, and slot 2 =
                                       its second buffer when world > 1 or, on one GPU, when
                                       the in-table Adam overlaps (see below)
  grads   float32 [2, V_pad, d]        local dense gradients (in, out)
  m, v    float32 [2, S, d]            Adam state of this rank's rows only

Row ownership: in table, rank r owns rows [r*S, (r+1)*S). Out table, cut into P pieces of
PL = V_pad / P rows: rank r owns sub-range r (SL = PL / world rows) of every piece; m[1], v[1]
hold those rows piece by piece. With P = 1 both tables have the same node-id ranges.

Per optimizer step, all collectives run over RCCL (torch.distributed 'nccl' on ROCm, xGMI),
per table (per piece for the out table):
  1. reduce-scatter(sum) of the gradient: rank r receives the global gradient of its rows;
  2. dense Adam on those rows only (dw_adam_dense): 1/world of the optimizer's HBM traffic;
  3. all-gather of the updated rows back into every rank's replica.

Overlapped form (``exchange_in`` / ``exchange_out_piece`` / ``exchange_out`` / ``sync``):
  * The in-table gradient is final after SGNS pass 1 (dw_sgns_walks_phase 1). ``exchange_in``
    runs the in-table's exchange on a side stream while the output-table phase (records sort +
    gather) still runs on the main stream. That phase reads the current in table, so the
    update goes into the idle buffer: copy own rows, Adam in place, all-gather into the
    buffer. The two buffers swap at ``sync``.
  * The output-table phase runs in row pieces (dw_sgns_walks_phase2_piece, sgns_phase2_pieces):
    piece p's gradient rows are final once its gather is done, and nothing in the phase reads
    the out table, so ``exchange_out_piece(p)`` exchanges piece p on the side stream while the
    gathers of the next pieces run. Only the last piece's exchange is exposed.
  * ``exchange_out`` exchanges the pieces not yet exchanged (all of them after an unpieced
    phase 2); ``sync`` makes the main stream wait for every all-gather before the next pass 1.
``step()`` is the same update done serially.

On one GPU there is nothing to exchange, but the in-table Adam (1/2 of the optimizer traffic) still
overlaps the output-table phase the same way (``overlap_in``, default on with the HIP Adam):
``exchange_in`` runs dw_adam_dense_to from the current in table into the idle buffer on the side
stream, and the radix sort of that phase leaves the HBM bandwidth it needs. The out table's Adam
is fused into the phase itself (``out_adam_spec``).

The Adam update is injectable (``adam_impl``), so the exchange logic can be tested with gloo
on the CPU (there the overlapped form runs its collectives synchronously). The default is the
HIP kernel, which refuses host tensors.
"""
import math
import os
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from shallow_encoders import _native


def adam_scalars(step: int, lr: float, betas, eps: float, weight_decay: float):
    """dw_adam_dense's scalar arguments for torch.optim.Adam step ``step`` (float64 on the host,
    as torch computes them): (1-b1, b2, 1-b2, sqrt(bias_correction2), -lr/bias_correction1,
    eps, weight_decay)."""
    beta1, beta2 = betas
    bias_correction1 = 1 - beta1 ** step
    bias_correction2 = 1 - beta2 ** step
    return (1 - beta1, beta2, 1 - beta2, bias_correction2 ** 0.5, -(lr / bias_correction1), eps,
            weight_decay)


# betas[1] values whose every step's sqrt(bias_correction2) c is PROVEN to give, through the
# reciprocal division of dw::div_bc2s (q = x RN(1/c); q + (x - c q) RN(1/c)), the IEEE quotient
# x / c for every fp32 x the replays divide (all 2^23 mantissas of [1, 2) and 0, per c; scaling
# by powers of two is exact there): scripts/microbench/div_proof.py on MI355X,
# profiles/r05_div_proof.jsonl (the random sample before it was not a proof). Other
# betas get no reciprocal (h[7] = 0): the kernels divide.
RECIPROCAL_PROVEN_BETA2 = (0.999, 0.99)


def bc2s_pairs(beta2: float) -> np.ndarray:
    """float32 [T, 2]: (sqrt(bias_correction2), RN(1 / it)) of steps 1..T as hist_row writes them,
    T the first step at which the first rounds to 1 (from there on y = 1 and q = x exactly)."""
    out = []
    t = 1
    while True:
        c = np.float32(adam_scalars(t, 1.0, (0.9, beta2), 1e-8, 0.0)[3])
        out.append((c, np.float32(1.0) / c))
        if c == np.float32(1.0) or t > 10_000_000:
            break
        t += 1
    return np.asarray(out, dtype=np.float32)


def hist_row(step: int, lr: float, betas, eps: float, weight_decay: float) -> np.ndarray:
    """float32[8]: adam_scalars as the kernels take them, then RN(1 / sqrt(bias_correction2))
    (the replays divide by the step's uniform sqrt(bias_correction2) through it: dw::div_bc2s)
    where betas[1] is proven for it (RECIPROCAL_PROVEN_BETA2), else 0 (divide)."""
    h = np.zeros(8, dtype=np.float32)
    h[:7] = np.asarray(adam_scalars(step, lr, betas, eps, weight_decay), dtype=np.float32)
    if float(betas[1]) in RECIPROCAL_PROVEN_BETA2:
        h[7] = np.float32(1.0) / h[3]
    return h


HIST_BOX_TAG = 0x58424457   # include/dw_hip.h DW_HIST_BOX_TAG


def _bits_in(x: np.ndarray, lo: float, hi: float) -> np.ndarray:
    """dw::in_bits: lo <= x <= hi on the float32 bits (x, lo, hi >= +0; a sign bit fails)."""
    b = x.astype(np.float32).view(np.uint32)
    lo_b = np.array(lo, dtype=np.float32).view(np.uint32)
    hi_b = np.array(hi, dtype=np.float32).view(np.uint32)
    return (b - lo_b) <= (hi_b - lo_b)   # uint32 wrap-around, as on the device


def hist_rows_in_box(rows: np.ndarray) -> np.ndarray:
    """bool per float32[8] history row: its scalars keep the lazy g = 0 replays in the box where
    sqrt and the division run without range scaling (dw_common.h, dw::replay_g0): weight_decay
    +0, the reciprocal present, eps in [2^-27, 1], sqrt(bias_correction2) in [2^-10, 1],
    1-beta1 and beta2 in [0, 1]."""
    r = np.ascontiguousarray(rows, dtype=np.float32).reshape(-1, 8)
    u = r.view(np.uint32)
    with np.errstate(over='ignore'):
        return ((u[:, 6] == 0) & (u[:, 7] != 0) & _bits_in(r[:, 5], 2.0 ** -27, 1.0)
                & _bits_in(r[:, 3], 2.0 ** -10, 1.0) & _bits_in(r[:, 0], 0.0, 1.0)
                & _bits_in(r[:, 1], 0.0, 1.0))


def hist_header(hist: np.ndarray, last: int) -> np.ndarray:
    """float32[8] row 0 of a lazy Adam history whose rows 1..last are written: the box tag, the
    first step b such that rows b..last are all in the box, and the frozen-parameter bound of
    those rows (include/dw_hip.h; dw_common.h, dw::frozen_el): [2] F = max |nstep| when every
    box row has the same eps and (1 - beta1)(1 + 2^-20) <= sqrt(beta2) (m then shrinks at least
    as fast as RN(sqrt(v)) over g = 0 steps), else +inf (no replay tail is frozen); [3] that
    eps; [4], [5] the rows' 1 - beta1 and beta2 when every box row has the same (the betas never
    changed: a frozen tail then steps m and v with them, no per-step history loads), else NaN."""
    ok = hist_rows_in_box(hist[1:last + 1])
    bad = np.flatnonzero(~ok)
    b = int(bad[-1]) + 2 if bad.size else 1
    h0 = np.zeros(8, dtype=np.float32)
    h0.view(np.uint32)[0] = HIST_BOX_TAG
    h0.view(np.int32)[1] = b
    h0[2] = np.inf
    h0[4] = h0[5] = np.nan
    rows = np.ascontiguousarray(hist[b:last + 1], dtype=np.float32).reshape(-1, 8)
    if rows.shape[0]:
        w1, b2 = rows[:, 0].astype(np.float64), rows[:, 1].astype(np.float64)
        eps = rows[:, 5]
        if (eps == eps[0]).all() and ((1.0 - w1) * (1.0 + 2.0 ** -20) <= np.sqrt(b2)).all():
            h0[2] = np.abs(rows[:, 4]).max()
            h0[3] = eps[0]
        bits = rows[:, :2].view(np.uint32)
        if (bits == bits[0]).all():
            h0[4], h0[5] = rows[0, 0], rows[0, 1]
    return h0


def hip_adam(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: int,
             lr: float, betas, eps: float, weight_decay: float, zero_grad: bool) -> None:
    """One dense Adam step on flat fp32 buffers with torch.optim.Adam's scalar math."""
    with torch.cuda.device(p.device):
        _native.call('dw_adam_dense', _native.ptr(p), _native.ptr(g), _native.ptr(m),
                     _native.ptr(v), p.numel(), *adam_scalars(step, lr, betas, eps, weight_decay),
                     1 if zero_grad else 0, _native.stream(p.device))


def hip_adam_to(p_src: torch.Tensor, p_dst: torch.Tensor, g: torch.Tensor, m: torch.Tensor,
                v: torch.Tensor, step: int, lr: float, betas, eps: float, weight_decay: float,
                zero_grad: bool, max_blocks: int = 0) -> None:
    """hip_adam reading the parameters from p_src and writing them to p_dst (dw_adam_dense_to);
    max_blocks > 0 caps the grid."""
    adam_to_scalars(p_src, p_dst, g, m, v, adam_scalars(step, lr, betas, eps, weight_decay),
                    zero_grad, max_blocks)


def adam_to_scalars(p_src: torch.Tensor, p_dst: torch.Tensor, g: torch.Tensor, m: torch.Tensor,
                    v: torch.Tensor, scalars: tuple, zero_grad: bool, max_blocks: int = 0) -> None:
    """dw_adam_dense_to with precomputed scalars (adam_scalars order), on the current stream."""
    assert p_src.numel() == p_dst.numel() == g.numel() == m.numel() == v.numel()
    with torch.cuda.device(p_src.device):
        _native.call('dw_adam_dense_to', _native.ptr(p_src), _native.ptr(p_dst), _native.ptr(g),
                     _native.ptr(m), _native.ptr(v), p_src.numel(), *scalars,
                     1 if zero_grad else 0, int(max_blocks), _native.stream(p_src.device))


# One GPU, in-table Adam on the side stream: its grid is sized so that it just finishes inside
# the overlapped phase (records sort + gather) and leaves the other CUs to that phase. The sort
# is latency-bound (~2 TB/s); a full-grid Adam takes every CU and doubles it, one capped to the
# rate it needs fills the unused bandwidth instead. Constants measured on MI355X at C3
# (profiles/r01_overlap_sweep.txt): the phase runs at ~5 TB/s of its byte model; one 256-thread
# Adam block moves ~22 GB/s next to it; 25% margin.
OVERLAP_PHASE_BPS = 5.0e12
ADAM_BLOCK_BPS = 22e9
# (round 6: 1.25 -> 1.375, 47 -> 51 blocks at C3: the capped Adam then ends inside the sort +
# gather window instead of ~0.1 ms after it; 6.85 -> 6.75 ms per step, 56 blocks 6.78, 42 7.20;
# profiles/r06_pipe_order_ab.txt)
OVERLAP_MARGIN = 1.375

# N > 1: out-table pieces exchanged behind the output-table phase; 8 keeps each collective at
# 1/8 of the table (64 MB at C3) while exposing only the last piece's exchange.
DEFAULT_OUT_PIECES = 8

# widths the owner passes (dw_sgns_owner_pass1/2, dw_sgns_owner_out_rows) are built for
OWNER_DIMS = ROWS_MAJOR_DIMS = (64, 128, 256, 512)


def overlap_adam_blocks(adam_bytes: float, overlap_bytes: Optional[float]) -> int:
    """Grid cap for an Adam of ``adam_bytes`` overlapping a phase of ``overlap_bytes``
    (0 = full grid, when no estimate is given)."""
    if not overlap_bytes:
        return 0
    t = overlap_bytes / OVERLAP_PHASE_BPS
    need = OVERLAP_MARGIN * adam_bytes / t / ADAM_BLOCK_BPS
    return int(min(8192, max(32, math.ceil(need))))


def force_collectives() -> bool:
    """DW_FORCE_COLLECTIVES=1 with a process group of one rank: take the N > 1 protocol
    (reduce-scatter / all-gather / all-reduce, side-stream overlap) anyway, so the RCCL flow of
    the multi-GPU step can be checked on a one-GPU box. Off by default: one rank then takes the
    one-device shortcuts (fused Adam, no collectives)."""
    return dist.is_initialized() and os.environ.get('DW_FORCE_COLLECTIVES') == '1'


class ShardedTables:
    """In/out embedding tables + dense gradients + node-range-sharded Adam state."""

    def __init__(self, vocab_size: int, dim: int, device, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 group=None, init_seed: Optional[int] = 0,
                 adam_impl: Optional[Callable] = None, overlap_in: Optional[bool] = None,
                 out_pieces: Optional[int] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.multi = self.world > 1 or force_collectives()   # collectives run
        self.V, self.d = int(vocab_size), int(dim)
        # out-table pieces: one per exchange pipelined behind the output-table phase (N > 1)
        self.P = int(out_pieces) if out_pieces else (DEFAULT_OUT_PIECES if self.multi else 1)
        if not 1 <= self.P <= 1024:
            raise ValueError('out_pieces must be in [1, 1024]')
        unit = self.world * self.P
        self.V_pad = int(math.ceil(self.V / unit)) * unit
        self.S = self.V_pad // self.world
        self.PL = self.V_pad // self.P          # rows per out-table piece
        self.SL = self.PL // self.world         # rows per rank per piece
        self.device = torch.device(device)
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.adam_impl = adam_impl or hip_adam
        self.step_count = 0
        self._cuda = self.device.type == 'cuda'
        if overlap_in is None:
            overlap_in = True
        # one GPU: the in-table Adam overlaps only with the HIP kernel (out of place)
        self.overlap_in = bool(overlap_in and not self.multi and self._cuda
                               and self.adam_impl is hip_adam)
        n_slots = 3 if (self.multi or self.overlap_in) else 2
        self.params = torch.zeros((n_slots, self.V_pad, self.d), dtype=torch.float32,
                                  device=self.device)
        self.grads = torch.zeros((2, self.V_pad, self.d), dtype=torch.float32, device=self.device)
        self.m = torch.zeros((2, self.S, self.d), dtype=torch.float32, device=self.device)
        self.v = torch.zeros_like(self.m)
        self.grad_shard = torch.empty_like(self.m) if self.multi else None
        self._cur_in = 0
        self._next_in = 0
        self._ag = []          # pending all-gathers / side-stream events (overlapped form)
        self._out_done = set()  # out-table pieces already exchanged this step
        self._side = (torch.cuda.Stream(self.device)
                      if (self._cuda and (self.multi or self.overlap_in)) else None)
        self._row_flags = None   # fused output-table Adam scratch (one device)
        if init_seed is not None:
            self.xavier_(init_seed)

    # ---- views -------------------------------------------------------------------------------
    @property
    def w_in(self) -> torch.Tensor:
        return self.params[self._cur_in, :self.V]

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
        """[start, end) rows of this rank's node range of the in table."""
        return self.rank * self.S, (self.rank + 1) * self.S

    def out_piece_rows(self, p: int):
        """[start, end) rows of out-table piece p, and of this rank's share of it."""
        a = p * self.PL
        return (a, a + self.PL), (a + self.rank * self.SL, a + (self.rank + 1) * self.SL)

    def state_rows(self, t: int, rank: Optional[int] = None) -> torch.Tensor:
        """Global row of each row of m[t] / v[t] (rank ``rank``'s rows of table t, in order;
        default this rank)."""
        r = self.rank if rank is None else int(rank)
        if t == 0:
            return torch.arange(r * self.S, (r + 1) * self.S)
        return torch.cat([torch.arange(p * self.PL + r * self.SL, p * self.PL + (r + 1) * self.SL)
                          for p in range(self.P)])

    def full_state(self):
        """(w_in, m_in, v_in, w_out, m_out, v_out), each the whole (V, d) table, on every rank:
        the tables are replicated; the Adam state shards (node ranges of the in table, piece
        sub-ranges of the out table) are all-gathered when N > 1 (collectives: every rank calls
        it). Between steps only (no exchange pending): bench.py's step check of the layout."""
        res = []
        for t in (0, 1):
            for st in (self.m[t], self.v[t]):
                if not self.multi:
                    full = torch.empty((self.V_pad, self.d), dtype=torch.float32,
                                       device=self.device)
                    full[self.state_rows(t).to(self.device)] = st
                else:
                    parts = torch.empty((self.world, self.S, self.d), dtype=torch.float32,
                                        device=self.device)
                    if dist.get_backend(self.group) == 'nccl':
                        dist.all_gather_into_tensor(parts.view(-1), st.reshape(-1),
                                                    group=self.group)
                    else:
                        dist.all_gather(list(parts.unbind(0)), st.clone(), group=self.group)
                    full = torch.empty((self.V_pad, self.d), dtype=torch.float32,
                                       device=self.device)
                    for r in range(self.world):
                        full[self.state_rows(t, r).to(self.device)] = parts[r]
                res.append(full[:self.V].clone())
        return (self.w_in.clone(), res[0], res[1], self.w_out.clone(), res[2], res[3])

    def xavier_(self, seed: int) -> None:
        """W2VBase init (model.py:26-27): U(-a, a), a = sqrt(6/(V+d)); identical on all ranks."""
        g = torch.Generator(device='cpu').manual_seed(int(seed))
        a = math.sqrt(6.0 / (self.V + self.d))
        for t in (self._cur_in, 1):
            w = torch.rand((self.V, self.d), generator=g) * (2 * a) - a
            self.params[t, :self.V].copy_(w)

    def load_(self, w_in: torch.Tensor, w_out: torch.Tensor) -> None:
        self.params[self._cur_in, :self.V].copy_(w_in)
        self.params[1, :self.V].copy_(w_out)

    def enable_exact(self, grad_scale: float) -> None:
        """The deterministic mode (word2vec/exact.py) for steps of this grad_scale: both
        gradient buffers get int64 fixed-point accumulators. One rank only: the replicated N > 1
        layout reduces float partial sums (use OwnerTables there)."""
        from shallow_encoders.word2vec import exact
        if self.multi:
            raise NotImplementedError('the deterministic mode covers the owner layout at N > 1 '
                                      '(OwnerTables), not the replicated one')
        self._exact = exact.Registry()
        # the in table's sums converted by its Adam (one streaming pass; _adam_both then
        # launches the two tables' updates separately)
        self._exact.ensure(0, self.grads[0], grad_scale,
                           adam=self._cuda and self.adam_impl is hip_adam)
        self._exact.ensure(1, self.grads[1], grad_scale)

    # ---- one table's exchange -------------------------------------------------------------------
    def _adam(self, p, g, t: int, zero_grad: bool) -> None:
        self.adam_impl(p, g, self.m[t].view(-1), self.v[t].view(-1), self.step_count, self.lr,
                       self.betas, self.eps, self.weight_decay, zero_grad)

    def _adam_both(self) -> None:
        """One device: Adam on both tables in place (one launch when they are adjacent)."""
        if (self.params.shape[0] == 2 and self._cur_in == 0
                and getattr(self, '_exact', None) is None):
            self.adam_impl(self.params.view(-1), self.grads.view(-1), self.m.view(-1),
                           self.v.view(-1), self.step_count, self.lr, self.betas, self.eps,
                           self.weight_decay, True)
            return
        self._adam(self.params[self._cur_in].view(-1), self.grads[0].view(-1), 0, True)
        self._adam(self.params[1].view(-1), self.grads[1].view(-1), 1, True)

    def _all_gather(self, dst: torch.Tensor, own: torch.Tensor, async_op: bool):
        nccl = dist.get_backend(self.group) == 'nccl'
        src = own.view(-1) if nccl else own.reshape(-1).clone()   # RCCL all-gather is in-place safe
        return dist.all_gather_into_tensor(dst.view(-1), src, group=self.group, async_op=async_op)

    def _exchange_in(self, src_slot: int, dst_slot: int, async_op: bool):
        """reduce-scatter grads[0] -> Adam on own rows of params[dst_slot] (starting from
        params[src_slot]) -> all-gather into params[dst_slot]; grads[0] ends zeroed.
        Returns the all-gather work handle when async_op."""
        a, b = self.shard_range()
        w = dist.reduce_scatter_tensor(self.grad_shard[0].view(-1), self.grads[0].view(-1),
                                       op=dist.ReduceOp.SUM, group=self.group,
                                       async_op=async_op)
        if async_op:
            w.wait()            # the current (side) stream waits for the reduce-scatter
        self.grads[0].zero_()
        own = self.params[dst_slot, a:b]
        if src_slot != dst_slot:
            own.copy_(self.params[src_slot, a:b])
        self._adam(own.view(-1), self.grad_shard[0].view(-1), 0, False)
        return self._all_gather(self.params[dst_slot], own, async_op)

    def _exchange_out_piece(self, p: int, async_op: bool):
        """The same for out-table piece p (rows out_piece_rows(p)); grads of the piece end
        zeroed. Returns the all-gather work handle when async_op."""
        (a, b), (oa, ob) = self.out_piece_rows(p)
        gp = self.grads[1, a:b]
        gs = self.grad_shard[1].view(self.P, self.SL, self.d)[p]
        w = dist.reduce_scatter_tensor(gs.view(-1), gp.reshape(-1), op=dist.ReduceOp.SUM,
                                       group=self.group, async_op=async_op)
        if async_op:
            w.wait()
        gp.zero_()
        own = self.params[1, oa:ob]
        self.adam_impl(own.view(-1), gs.view(-1),
                       self.m[1].view(self.P, self.SL, self.d)[p].view(-1),
                       self.v[1].view(self.P, self.SL, self.d)[p].view(-1), self.step_count,
                       self.lr, self.betas, self.eps, self.weight_decay, False)
        return self._all_gather(self.params[1, a:b], own, async_op)

    # ---- serial step ------------------------------------------------------------------------------
    def step(self) -> None:
        """Exchange gradients, update this rank's rows, gather parameters; grads end zeroed."""
        self.sync()
        self.step_count += 1
        if not self.multi:
            self._adam_both()
            return
        self._exchange_in(self._cur_in, self._cur_in, False)
        for p in range(self.P):
            self._exchange_out_piece(p, False)

    # ---- overlapped step --------------------------------------------------------------------------
    def _on_side(self, fn) -> None:
        """Run fn on the side stream after the work enqueued so far on the current stream (CPU:
        now). fn returns a work handle / event that ``sync`` waits for, or None."""
        if not self._cuda:
            fn(False)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            self._side.wait_event(ev)
            w = fn(True)
            if w is not None:
                self._ag.append(w)

    def exchange_in(self, overlap_bytes: Optional[float] = None) -> None:
        """Call right after SGNS pass 1 is enqueued (g_in final): the in-table update starts on a
        side stream while the output-table phase runs on the current stream. ``overlap_bytes``
        (one GPU): HBM bytes of that phase (sgns_phase_bytes sort + pass2), to size the Adam's
        grid (overlap_adam_blocks); None = full grid."""
        self.step_count += 1
        self._out_done = set()
        if not self.multi and not self.overlap_in:
            return                              # exchange_out does the Adam
        self._next_in = 2 - self._cur_in
        if not self.multi:
            def adam_to(_async):
                # (the deterministic mode's update reads and clears the 8-B sums instead of g)
                per = 4 * 7 + (8 if getattr(self, '_exact', None) is not None else 0)
                blocks = overlap_adam_blocks(self.V_pad * self.d * per, overlap_bytes)
                hip_adam_to(self.params[self._cur_in], self.params[self._next_in],
                            self.grads[0], self.m[0], self.v[0], self.step_count, self.lr,
                            self.betas, self.eps, self.weight_decay, True, blocks)
                done = torch.cuda.Event()
                done.record(self._side)
                return done
            self._on_side(adam_to)
            return
        self._on_side(lambda a: self._exchange_in(self._cur_in, self._next_in, a))

    def out_pieces_spec(self):
        """(n_pieces, piece_rows) for sgns_phase2_pieces."""
        return self.P, self.PL

    def exchange_out_piece(self, p: int) -> None:
        """Call right after the gather of out-table piece p is enqueued (its gradient rows
        final): its reduce-scatter / Adam / all-gather run on the side stream while the next
        pieces' gathers run. One GPU: nothing to exchange (exchange_out does the Adam)."""
        if not self.multi:
            return
        if p in self._out_done:
            raise RuntimeError(f'out-table piece {p} exchanged twice in one step')
        self._out_done.add(p)
        self._on_side(lambda a: self._exchange_out_piece(p, a))

    def can_fuse_out_adam(self) -> bool:
        """The output table's Adam can run inside SGNS phase 2: one device, HIP Adam."""
        return not self.multi and self._cuda and self.adam_impl is hip_adam

    def out_adam_spec(self) -> Optional[dict]:
        """For SGNS phase 2 with the output table's Adam fused in (sgns_accumulate out_adam=):
        call after exchange_in (this step's scalars), then exchange_out(fused_out=True). None
        where the fusion does not apply (can_fuse_out_adam)."""
        if not self.can_fuse_out_adam():
            return None
        if self.step_count < 1:
            raise RuntimeError('out_adam_spec() before exchange_in(): no step to fuse')
        if self._row_flags is None:
            self._row_flags = torch.zeros(self.V_pad, dtype=torch.uint8, device=self.device)
        return {'m': self.m[1], 'v': self.v[1], 'flags': self._row_flags,
                'scalars': adam_scalars(self.step_count, self.lr, self.betas, self.eps,
                                        self.weight_decay)}

    def exchange_out(self, fused_out: bool = False) -> None:
        """Call right after SGNS phase 2 is enqueued (g_out final): exchanges the out-table
        pieces exchange_out_piece has not. ``fused_out``: phase 2 already applied the output
        table's Adam (out_adam_spec, one GPU)."""
        if not self.multi:
            if self.overlap_in:
                if not fused_out:       # the in table is done on the side stream (exchange_in)
                    self._adam(self.params[1].view(-1), self.grads[1].view(-1), 1, True)
            elif fused_out:
                self._adam(self.params[self._cur_in].view(-1), self.grads[0].view(-1), 0, True)
            else:
                self._adam_both()
            return
        for p in range(self.P):
            if p not in self._out_done:
                self.exchange_out_piece(p)

    def sync(self) -> None:
        """The current stream waits for pending all-gathers; the new in table becomes current.
        Call before the next SGNS pass 1 (and before reading the tables)."""
        for w in self._ag:
            if isinstance(w, torch.cuda.Event):
                torch.cuda.current_stream(self.device).wait_event(w)
            else:
                w.wait()
        self._ag = []
        self._cur_in = self._next_in


def replicated_step(tables: ShardedTables, walks: torch.Tensor, context_radius: int,
                    neg_samples: int, *, seed: int, noise_offset: int, grad_scale: float,
                    loss_acc: torch.Tensor, status: torch.Tensor, scatter: str = 'sorted',
                    fuse_out_adam: bool = True, pieces: bool = False,
                    after_pass1: Optional[Callable[[], None]] = None,
                    after_phase2: Optional[Callable[[], None]] = None) -> None:
    """One training step of ``tables`` over the batch ``walks`` — bench.py's step at N = 1 (and
    the replicated layout at N > 1), also run at full C3 size by tests/test_gpu_c3_step.py:

      SGNS pass 1 (g_in final; device negatives when ``noise`` is not given)
      -> in-table Adam (N = 1: dw_adam_dense_to into the idle buffer on the side stream, grid
         sized to the output-table phase; N > 1: reduce-scatter / Adam / all-gather)
      -> output-table phase with the out table's Adam fused (N = 1, records path) or in pieces
         exchanged behind the gathers (N > 1, ``pieces``)
      -> remaining exchanges, then the main stream joins the side stream.

    ``after_pass1`` / ``after_phase2``: host callbacks at those two points of the enqueue order
    (bench.py records events and hands the walk buffer back there)."""
    from shallow_encoders.word2vec.sgns import (sgns_accumulate, sgns_phase2_pieces,
                                                sgns_phase_bytes)
    n, L = walks.shape
    R, K = int(context_radius), int(neg_samples)
    kw = dict(walks=walks, context_radius=R, noise=None, seed=seed, noise_offset=noise_offset,
              grad_scale=grad_scale, loss_acc=loss_acc, status=status, scatter=scatter)
    fuse = fuse_out_adam and scatter == 'sorted' and tables.can_fuse_out_adam()
    pb = sgns_phase_bytes(n, L, R, K, tables.d, tables.V, scatter, fuse)
    sgns_accumulate(tables.w_in, tables.w_out, tables.g_in, tables.g_out, K, phase=1, **kw)
    if after_pass1 is not None:
        after_pass1()
    tables.exchange_in(overlap_bytes=pb['sort'] + pb['pass2'])
    spec = tables.out_adam_spec() if fuse else None
    if pieces:
        n_pieces, rows = tables.out_pieces_spec()
        sgns_phase2_pieces(tables.w_in, tables.g_out, K, walks=walks, context_radius=R,
                           n_pieces=n_pieces, piece_rows=rows,
                           on_piece=tables.exchange_out_piece, status=status, scatter=scatter)
    else:
        sgns_accumulate(tables.w_in, tables.w_out, tables.g_in, tables.g_out, K, phase=2,
                        out_adam=spec, **kw)
    if after_phase2 is not None:
        after_phase2()
    tables.exchange_out(fused_out=spec is not None)
    tables.sync()


class OwnerTables:
    """N > 1, owner-computes layout (the multi-GPU default of bench.py).

    The output ("context") table never crosses ranks: rank r holds only the rows o with
    o % world == r (local row o // world; interleaved ownership spreads R-MAT's low-id hubs over
    all ranks), with their Adam state, and updates them itself. Every rank forms the windows of
    the WHOLE global batch (walks are keyed by the global walk id, so it generates them all)
    and computes only the output slots whose row it owns (dw_sgns_owner_pass1 / _pass2); summed
    over the ranks that is exactly the single-device computation, so this is DDP-equivalent
    training of the global batch with no output-table collective at all.

    The in table is replicated and double-buffered as in ShardedTables: each rank's pass 1 adds
    the partial centre gradient of its owned slots into the dense g_in, and ``exchange_in``
    reduce-scatters it by node-id range (rank r owns rows [r*S, (r+1)*S)), applies Adam to the
    own rows and all-gathers them into the idle buffer, on a side stream behind the
    output-table phase. Per step that is the in table's 2 x V*d*4 B over xGMI and nothing else
    (ShardedTables moves both tables: twice that).

      params_in  float32 [2, V_pad, d]   replicated in table, two buffers
      g_in       float32 [V_pad, d]      partial (this rank's slots) centre gradient
      m_in, v_in float32 [S, d]          Adam state of the own in-table rows
      w_out      float32 [S, d]          local out-table slice (global row r + world*j)
      g_out      float32 [S, d]          its gradient (zero between steps)
      m_out, v_out float32 [S, d]        its Adam state

    V_pad = V rounded up to a multiple of world, S = V_pad / world. ``adam_impl`` is injectable
    as in ShardedTables (CPU tests over gloo).
    """

    def __init__(self, vocab_size: int, dim: int, device, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 group=None, init_seed: Optional[int] = 0,
                 adam_impl: Optional[Callable] = None, emulate_world: Optional[int] = None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # emulate_world (one process, measurement only: bench.py --emulate-world): act as rank 0
        # of that many ranks — the same per-rank kernels and Adam shares, no collectives (the
        # in-table rows of the other ranks are then never refreshed)
        self.emulated = bool(emulate_world) and self.world == 1
        if self.emulated:
            self.world, self.rank = int(emulate_world), 0
        # collectives run (N > 1, or one rank with DW_FORCE_COLLECTIVES=1); never emulated
        self.multi = (self.world > 1 or force_collectives()) and not self.emulated
        self.V, self.d = int(vocab_size), int(dim)
        self.V_pad = int(math.ceil(self.V / self.world)) * self.world
        self.S = self.V_pad // self.world
        self.device = torch.device(device)
        self.lr, self.betas, self.eps, self.weight_decay = lr, tuple(betas), eps, weight_decay
        self.adam_impl = adam_impl or hip_adam
        self.step_count = 0
        self._cuda = self.device.type == 'cuda'
        if self._cuda and self.d not in OWNER_DIMS:
            # the owner passes' kernels (k_sgns_g16 owner / COEFIN forms, k_out_rows) exist for
            # these widths only: refuse here rather than fail inside a step
            raise ValueError(f'the owner layout needs d in {OWNER_DIMS} (got {self.d}); use '
                             f'ShardedTables (the replicated layout) for other widths')
        f32 = dict(dtype=torch.float32, device=self.device)
        self._alloc_in(f32)
        self.w_out = torch.zeros((self.S, self.d), **f32)
        self.g_out = torch.zeros_like(self.w_out)
        self.m_out = torch.zeros_like(self.w_out)
        self.v_out = torch.zeros_like(self.w_out)
        self._flags = torch.zeros(self.S, dtype=torch.uint8, device=self.device)
        self._cur_in = 0
        self._next_in = 0
        self._ag = []
        self._overlap_bytes = None
        self._side = torch.cuda.Stream(self.device) if self._cuda else None
        if init_seed is not None:
            self.xavier_(init_seed)

    def _alloc_in(self, f32: dict) -> None:
        """The in table (two buffers), its dense partial gradient and the own rows' Adam state."""
        self.params_in = torch.zeros((2, self.V_pad, self.d), **f32)
        self.grads_in = torch.zeros((self.V_pad, self.d), **f32)
        self.m_in = torch.zeros((self.S, self.d), **f32)
        self.v_in = torch.zeros_like(self.m_in)
        self.grad_shard = (torch.empty_like(self.m_in) if self.multi
                           else None)

    # ---- views -------------------------------------------------------------------------------
    @property
    def w_in(self) -> torch.Tensor:
        return self.params_in[self._cur_in, :self.V]

    @property
    def w_in_raw(self) -> torch.Tensor:
        """The in table as the SGNS passes read it (the same as w_in here)."""
        return self.params_in[self._cur_in, :self.V]

    @property
    def g_in(self) -> torch.Tensor:
        return self.grads_in[:self.V]

    def shard_range(self):
        """[start, end) rows of this rank's node range of the in table."""
        return self.rank * self.S, (self.rank + 1) * self.S

    def out_rows(self) -> torch.Tensor:
        """Global row of each local out-table row (r, r + world, ...; some >= V are padding)."""
        return torch.arange(self.S) * self.world + self.rank

    def xavier_(self, seed: int) -> None:
        """The same initial tables as ShardedTables.xavier_ (model.py:26-27), this rank's slice of
        the out table."""
        g = torch.Generator(device='cpu').manual_seed(int(seed))
        a = math.sqrt(6.0 / (self.V + self.d))
        w_in = torch.rand((self.V, self.d), generator=g) * (2 * a) - a
        w_out = torch.rand((self.V, self.d), generator=g) * (2 * a) - a
        self.load_(w_in, w_out)

    def load_(self, w_in: torch.Tensor, w_out: torch.Tensor) -> None:
        """Set the tables from full (V, d) tensors (every rank passes the same ones)."""
        self.params_in[self._cur_in, :self.V].copy_(w_in)
        rows = self.out_rows()
        keep = rows < self.V
        self.w_out.zero_()
        self.w_out[keep] = w_out[rows[keep]].to(self.device)

    def enable_exact(self, grad_scale: float) -> None:
        """The deterministic mode (word2vec/exact.py) for steps of this grad_scale: g_out and
        g_in get int64 fixed-point accumulators. N > 1: each rank's centre sums stay integers,
        are reduce-scattered as int64 (exact) and converted on the owning rank — the tables are
        bit-identical to one rank's."""
        from shallow_encoders.word2vec import exact
        if getattr(self, 'lazy', False) or type(self) is not OwnerTables:
            raise NotImplementedError('the deterministic mode covers the dense OwnerTables')
        if self.emulated:
            raise NotImplementedError('the deterministic mode needs the real collectives')
        self._exact = exact.Registry()
        self._exact.ensure(0, self.grads_in, grad_scale, defer=self.multi)
        self._exact.ensure(1, self.g_out, grad_scale)
        self._shard64 = torch.empty((self.S, self.d), dtype=torch.int64, device=self.device) \
            if self.multi else None

    def full_w_out(self) -> torch.Tensor:
        """The whole (V, d) out table, gathered from every rank's slice (collective when N > 1)."""
        if self.emulated:
            raise RuntimeError('an emulated rank holds only its own slice')
        if not self.multi:
            return self.w_out[:self.V].clone()
        parts = torch.empty((self.world, self.S, self.d), dtype=torch.float32, device=self.device)
        if dist.get_backend(self.group) == 'nccl':
            dist.all_gather_into_tensor(parts.view(-1), self.w_out.view(-1), group=self.group)
        else:
            dist.all_gather(list(parts.unbind(0)), self.w_out.clone(), group=self.group)
        # local row j of rank r is global row r + world * j
        return parts.transpose(0, 1).reshape(self.V_pad, self.d)[:self.V].clone()

    def out_state_full(self):
        """(m, v) of the out table as full (V, d) tensors (gathered, as full_w_out)."""
        res = []
        for t in (self.m_out, self.v_out):
            w, self.w_out = self.w_out, t
            try:
                res.append(self.full_w_out())
            finally:
                self.w_out = w
        return tuple(res)

    def in_state_full(self):
        """(m, v) of the in table as full (V, d) tensors: the node-range shards all-gathered
        (collective when N > 1)."""
        if self.emulated:
            raise RuntimeError('an emulated rank holds only its own shard')
        if not self.multi:
            return self.m_in[:self.V].clone(), self.v_in[:self.V].clone()
        res = []
        for t in (self.m_in, self.v_in):
            full = torch.empty((self.world * self.S, self.d), dtype=torch.float32,
                               device=self.device)
            if dist.get_backend(self.group) == 'nccl':
                dist.all_gather_into_tensor(full.view(-1), t.reshape(-1), group=self.group)
            else:
                dist.all_gather(list(full.view(self.world, self.S, self.d).unbind(0)), t.clone(),
                                group=self.group)
            res.append(full[:self.V].clone())
        return tuple(res)

    def full_state(self):
        """(w_in, m_in, v_in, w_out, m_out, v_out), each the whole (V, d) table as the dense
        update holds it, on every rank (collectives when N > 1; lazy rows flushed first):
        bench.py's step self-check."""
        w_in = self.w_in.clone()
        m_in, v_in = self.in_state_full()
        m_out, v_out = self.out_state_full()
        return w_in, m_in, v_in, self.full_w_out(), m_out, v_out

    # ---- the step ------------------------------------------------------------------------------
    def _adam(self, p, g, m, v, zero_grad: bool) -> None:
        self.adam_impl(p, g, m, v, self.step_count, self.lr, self.betas, self.eps,
                       self.weight_decay, zero_grad)

    def _adam_own(self, src: torch.Tensor, dst: torch.Tensor, g: torch.Tensor) -> None:
        """Adam on the own in-table rows from the current buffer into the idle one: one
        out-of-place HIP pass (dw_adam_dense_to, grid capped to the overlapped phase) or copy +
        the injected update."""
        if self.adam_impl is hip_adam:
            blocks = overlap_adam_blocks(self.S * self.d * 4 * 7, self._overlap_bytes)
            adam_to_scalars(src, dst, g, self.m_in, self.v_in,
                            adam_scalars(self.step_count, self.lr, self.betas, self.eps,
                                         self.weight_decay), False, blocks)
            return
        dst.copy_(src)
        self._adam(dst.view(-1), g.reshape(-1), self.m_in.view(-1), self.v_in.view(-1), False)

    def _exchange_in(self, async_op: bool):
        """reduce-scatter g_in -> Adam on own rows of the idle buffer -> all-gather into it;
        g_in ends zeroed. One rank: Adam over the whole in table into the idle buffer."""
        src, dst = self.params_in[self._cur_in], self.params_in[self._next_in]
        if self.world == 1 and not self.multi:
            dst.copy_(src)
            self._adam(dst.view(-1), self.grads_in.view(-1), self.m_in.view(-1),
                       self.v_in.view(-1), True)
            return None
        a, b = self.shard_range()
        if self.emulated:   # this rank's share of the work, without the collectives
            self._adam_own(src[a:b], dst[a:b], self.grads_in[a:b])
            self.grads_in.zero_()
            return None
        fx = self._exact.get(0) if getattr(self, '_exact', None) is not None else None
        if fx is not None:   # deterministic: the integer centre sums, reduced exactly
            w = dist.reduce_scatter_tensor(self._shard64.view(-1), fx.acc.view(-1),
                                           op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=async_op)
            if async_op:
                w.wait()
            fx.acc.zero_()
            fx.convert(acc=self._shard64, out=self.grad_shard)
        else:
            w = dist.reduce_scatter_tensor(self.grad_shard.view(-1), self.grads_in.view(-1),
                                           op=dist.ReduceOp.SUM, group=self.group,
                                           async_op=async_op)
            if async_op:
                w.wait()
        self.grads_in.zero_()
        own = dst[a:b]
        self._adam_own(src[a:b], own, self.grad_shard)
        nccl = dist.get_backend(self.group) == 'nccl'
        send = own.view(-1) if nccl else own.reshape(-1).clone()
        return dist.all_gather_into_tensor(dst.view(-1), send, group=self.group,
                                           async_op=async_op)

    def exchange_in(self, overlap_bytes: Optional[float] = None) -> None:
        """Call right after pass 1 is enqueued (this rank's g_in final): the in-table update
        runs on a side stream into the idle buffer while the output-table phase reads the
        current one. Also starts the step (the Adam step count). ``overlap_bytes``: HBM bytes of
        that phase, to cap the own-rows Adam's grid (overlap_adam_blocks); None = full grid."""
        self.step_count += 1
        self._overlap_bytes = overlap_bytes
        self._next_in = 1 - self._cur_in
        if not self._cuda:
            self._exchange_in(False)
            return
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self._side):
            self._side.wait_event(ev)
            w = self._exchange_in(True)
            done = torch.cuda.Event()
            done.record(self._side)
            self._ag.append(w if w is not None else done)
            if w is not None:
                self._ag.append(done)

    def can_fuse_out_adam(self) -> bool:
        return self._cuda and self.adam_impl is hip_adam

    def out_adam_spec(self) -> Optional[dict]:
        """The slice's Adam for sgns_owner_pass2 (after exchange_in: this step's scalars); None
        where it cannot be fused (then call out_step after the gradient is in g_out)."""
        if not self.can_fuse_out_adam():
            return None
        if self.step_count < 1:
            raise RuntimeError('out_adam_spec() before exchange_in(): no step to fuse')
        return {'m': self.m_out, 'v': self.v_out, 'flags': self._flags,
                'scalars': adam_scalars(self.step_count, self.lr, self.betas, self.eps,
                                        self.weight_decay)}

    def out_step(self) -> None:
        """Unfused: Adam on the local slice from g_out (zeroed)."""
        self._adam(self.w_out.view(-1), self.g_out.view(-1), self.m_out.view(-1),
                   self.v_out.view(-1), True)

    def sync(self) -> None:
        """The current stream waits for the in-table update; the new in table becomes current.
        Call before the next pass 1 (and before reading w_in)."""
        for w in self._ag:
            if isinstance(w, torch.cuda.Event):
                torch.cuda.current_stream(self.device).wait_event(w)
            else:
                w.wait()
        self._ag = []
        self._cur_in = self._next_in


def owner_step(tables: 'OwnerTables', walks: torch.Tensor, context_radius: int,
               neg_samples: int, *, seed: int, noise_offset: int, grad_scale: float,
               loss_acc: torch.Tensor, status: torch.Tensor,
               overlap_bytes: Optional[float] = None) -> int:
    """One owner-computes training step over the global batch ``walks`` (every rank passes the
    same walks): pass 1 (owned slots) -> in-table exchange on the side stream -> pass 2 with the
    slice's Adam fused -> sync. Returns this rank's record count."""
    from shallow_encoders.word2vec.sgns import sgns_owner_pass1, sgns_owner_pass2
    sgns_owner_pass1(tables.w_in, tables.w_out, tables.grads_in, neg_samples, walks=walks,
                     context_radius=context_radius, owner=tables.rank, n_owners=tables.world,
                     vocab_size=tables.V, seed=seed, noise_offset=noise_offset,
                     grad_scale=grad_scale, loss_acc=loss_acc, status=status)
    tables.exchange_in(overlap_bytes)
    spec = tables.out_adam_spec()
    n = sgns_owner_pass2(tables.w_in, tables.w_out, tables.g_out, neg_samples, walks=walks,
                         context_radius=context_radius, out_adam=spec, status=status,
                         read_count=tables.world > 1)
    if n is None:   # one owner keeps every slot (no count readback)
        n = walks.shape[0] * (walks.shape[1] - 2 * context_radius) * 2 * context_radius * (
            1 + neg_samples)
    if spec is None:
        tables.out_step()
    tables.sync()
    return n


HIST_CAP0 = 1024   # initial rows of OwnerLazyTables' Adam-scalar history (doubled on demand)
HIST_AHEAD = 256   # history rows written per host-to-device copy (begin_step)


def hip_rows_adam(p: torch.Tensor, m: torch.Tensor, v: torch.Tensor, last: torch.Tensor,
                  rows: Optional[torch.Tensor], n_dev: Optional[torch.Tensor], n_max: int,
                  g_rows: Optional[torch.Tensor], hist: torch.Tensor, step: int,
                  pending: Optional[torch.Tensor] = None, grad_by_row: bool = False) -> None:
    """dw_adam_rows on [n_table, d] tables (see include/dw_hip.h); ``pending``: the rows-major
    step's uint8 marks (settled and cleared on the listed rows); ``grad_by_row``: ``g_rows`` is
    the table's dense gradient, row r's step reads (and clears) g_rows[r]."""
    with torch.cuda.device(p.device):
        _native.call('dw_adam_rows', _native.ptr(p), _native.ptr(m), _native.ptr(v),
                     _native.ptr(last), _native.ptr(pending), p.shape[0], p.shape[1],
                     _native.ptr(rows), _native.ptr(n_dev), int(n_max), _native.ptr(g_rows),
                     1 if grad_by_row else 0, _native.ptr(hist), int(step),
                     _native.stream(p.device))


class OwnerLazyTables(OwnerTables):
    """Owner-computes layout with the touched-row in-table exchange (``bench.py --in-exchange
    lazy``): SURVEY.md §8e's "throughput mode" — traffic proportional to the rows a step touches,
    not to V — kept exact.

    The out table is OwnerTables' owner slice. The in table, its Adam state and the step each row
    is current to (``last_in``) are replicated on every rank. A step reads and updates only the
    in rows of the global batch's centres, U (every rank holds the same walks, so every rank
    builds the same sorted U). Every other row has g = 0 for the step, and torch's Adam with
    g = 0 is a fixed recurrence in (p, m, v): it is deferred and replayed exactly (dw_adam_rows:
    the same adam_elem, step by step) when the row is next in U or the table is read (``flush``;
    the ``w_in`` property flushes). Per step (owner_lazy_step):
      begin_step        records the step's Adam scalars (the replays use them later);
      prepare           the batch's centre order and U (dw_sgns_owner_prepare);
      catch_up          the rows of U replay their missed steps, up to step - 1;
      catch_up_out      (lazy_out) the out rows the batch's slots reference, likewise;
      (pass 1)          the partial centre gradient of the owned slots into g_in (rows of U);
      exchange_touched  G = g_in[U] (those rows cleared) and all-reduce(SUM) of G on a side
                        stream while pass 2 runs: |U| x d x 4 B per step instead of the dense
                        reduce-scatter + all-gather of 2 x V x d x 4 B;
      (pass 2)          the out slice's records with its Adam fused, as OwnerTables;
      update_touched    step t on the rows of U with G, on every rank from identical inputs, so
                        the replicas stay bit-identical.
    On the CPU (gloo tests, ``adam_impl`` injected) the same protocol runs with torch ops, and
    ``set_touched`` stands in for ``prepare``.

      params_in  float32 [1, V_pad, d]  replicated in table
      m_in, v_in float32 [V_pad, d]     its Adam state, replicated
      last_in    int32 [V_pad]          step each row is current to

    ``lazy_out`` (HIP only): the out slice's Adam is lazy too — pass 2 updates only the rows its
    records touch, each after replaying its deferred g = 0 steps (dw_sgns_owner_pass2_lazy;
    ``last_out`` int32 [S]); ``flush`` brings both tables current. It pays where a step's
    records touch a small share of the slice (C3 at the reference's 64-walk batches: ~23% of
    the rows), so the dense out-table Adam (V·d·4 B x 7 per step) is not paid for the rest.
    """

    def __init__(self, *args, lazy_out: bool = False, **kwargs):
        self.lazy_out = bool(lazy_out)
        super().__init__(*args, **kwargs)
        self.lazy_out = self.lazy_out and self._hip()
        self.last_out = (torch.zeros(self.S, dtype=torch.int32, device=self.device)
                         if self.lazy_out else None)
        self._claim_out = torch.zeros_like(self.last_out) if self.lazy_out else None
        # placed records: every row's slot count of the step (+ one zero past the rows), cleared
        # by the lazy gather (dw_sgns_owner_out_catch_up / _pass2_lazy)
        self._count_out = (torch.zeros(self.S + 1, dtype=torch.int32, device=self.device)
                           if self.lazy_out else None)
        self._betas0 = tuple(self.betas)
        self._out_rows = None
        self._n_out = torch.zeros(1, dtype=torch.int64, device=self.device)
        # the records placed by the claim (no sort before the lazy gather; N > 1: each rank
        # places its own o % W slots into its slice's row segments)
        self.place = self.lazy_out
        # any step with weight decay: the p-only catch-up no longer holds
        self._wd_seen = False
        # placed records: the rows-major step (dw_sgns_owner_out_rows) reads and writes each
        # touched out row once; the catch-up -> pass 1 -> lazy gather sequence otherwise (the
        # tests set these attributes to compare the forms)
        self.rows_major = self.place
        # the rows-major step leaves the rows it steps pending (m, v at the step, p one behind
        # for the centre pass; pend_out[row] = 1); the next replay or a flush settles them
        self.pend_out = (torch.zeros(self.S, dtype=torch.uint8, device=self.device)
                         if self.lazy_out else None)
        self._pend_dirty = False   # some out row may be pending
        self._rows_step = False    # this step goes rows-major (set by catch_up_out)
        # the pipelined steps (owner_lazy_steps): the odd steps' row counts, touched lists and
        # catch-up lists (allocated by _pipe_alloc, outside any capture)
        self._count_out2 = None
        self._pipe = None

    def rows_major_ok(self, context_radius: int, neg_samples: int) -> bool:
        """The rows-major step applies: placed records, d one of the widths its kernels are
        built for (dw_sgns_owner_out_rows and the COEFIN pass 1: 64, 128, 256, 512),
        2R(1+K) <= 64 (the deterministic mode included: both kernels have its integer sums).
        Other widths keep the catch-up -> pass 1 -> lazy gather sequence."""
        return (self.rows_major and self.place and self.d in ROWS_MAJOR_DIMS
                and 2 * int(context_radius) * (1 + int(neg_samples)) <= 64)

    def enable_exact(self, grad_scale: float) -> None:
        """The deterministic mode (word2vec/exact.py) with the HIP lazy Adam of both tables:
        grads_in and g_out get int64 fixed-point accumulators, so the rows-major step sums every
        out row's terms (k_out_rows) and every centre's (the COEFIN pass) as integers — the same
        sums whatever order the claim's atomics ranked the records in — and the tables are
        bit-identical run to run, and to the dense deterministic step's (the lazy replays are
        the dense g = 0 steps bit for bit). N > 1: each rank's centre sums stay integers
        (DW_EXACT_DEFER), the touched rows' sums are all-reduced as int64 (exact) and converted
        alike on every rank — the tables equal one rank's bit for bit."""
        from shallow_encoders.word2vec import exact
        if not self._hip() or not self.lazy_out:
            raise NotImplementedError('the lazy deterministic mode covers the HIP lazy Adam of '
                                      'both tables (lazy_out)')
        if self.emulated and self.world > 1:
            raise NotImplementedError('the deterministic mode needs the real collectives')
        self._exact = exact.Registry()
        self._exact.ensure(0, self.grads_in, grad_scale, defer=self.multi)
        self._exact.ensure(1, self.g_out, grad_scale)

    def pipeline_ok(self, context_radius: int, neg_samples: int) -> bool:
        """owner_lazy_steps pipelines the steps: one rank, the HIP lazy Adam of both tables and
        the rows-major out step."""
        return (self.lazy_out and not self.multi and self._hip()
                and self.rows_major_ok(context_radius, neg_samples))

    def _pipe_alloc(self, n_walks: int, walk_length: int, context_radius: int,
                    neg_samples: int, n_steps: int = 64) -> None:
        """The pipelined steps' second buffers and their counter ring (one (|U|, fresh) pair per
        step of an owner_lazy_steps call; before a capture: a graph must not allocate)."""
        from shallow_encoders.word2vec.sgns import workspace_for
        n = max(n_walks * (walk_length - 2 * int(context_radius)), 1)
        for slot in (0, 1):
            workspace_for(n, 2 * int(context_radius), int(neg_samples), self.V, self.device,
                          local_rows=self.S, slot=slot)
        if self._count_out2 is None:
            self._count_out2 = torch.zeros_like(self._count_out)
        if self._claim_in is None:
            self._claim_in = torch.zeros(self.V_pad, dtype=torch.int32, device=self.device)
        p = self._pipe
        if p is None or p['touched'][0].numel() < n or p['ctr'].shape[0] < n_steps:
            i32 = dict(dtype=torch.int32, device=self.device)
            i64 = dict(dtype=torch.int64, device=self.device)
            self._pipe = {'touched': [torch.empty(n, **i32) for _ in range(2)],
                          'fresh': [torch.empty(n, **i32) for _ in range(2)],
                          # step k's [|U|, fresh] counters, cleared by one memset per call
                          'ctr': torch.zeros((max(n_steps, 64), 2), **i64)}
        if self._touched is None or self._touched.numel() < n:
            self._touched = torch.empty(n, dtype=torch.int32, device=self.device)

    def _touch_ahead(self, walks: torch.Tensor, context_radius: int, step: int,
                     slot: int, ctr: torch.Tensor) -> None:
        """The pipelined step ``step``'s in rows, while step - 1 may still run: its distinct
        centres U (touched list ``slot``, its count ctr[0]) and, of them, those that were not
        centres of step - 1 (the fresh list, count ctr[1]) replayed up to step - 1 — nothing of
        step - 1 writes those rows. ``ctr`` is zero on entry (the call's counter ring)."""
        p = self._pipe
        with torch.cuda.device(self.device):
            _native.call('dw_sgns_owner_touch_claim', _native.ptr(walks), walks.shape[0],
                         walks.shape[1], int(context_radius), self.V,
                         _native.ptr(self._claim_in), int(step),
                         _native.ptr(p['touched'][slot]), _native.ptr(ctr[0:1]),
                         _native.ptr(p['fresh'][slot]), _native.ptr(ctr[1:2]), 1,
                         _native.stream(self.device))
        n_max = walks.shape[0] * (walks.shape[1] - 2 * int(context_radius))
        hip_rows_adam(self.params_in[0], self.m_in, self.v_in, self.last_in, p['fresh'][slot],
                      ctr[1:2], n_max, None, self._hist, int(step) - 1)

    def out_flags(self) -> int:
        """dw_sgns_owner_out_catch_up / _pass2_lazy flags of the current step: 1 = place the
        records (one rank), 2 = the catch-up replays p only (no weight decay so far), 4 = the
        betas never changed (the gather's m, v replays need no history loads)."""
        if not self.lazy_out:
            return 0
        p_only = not self._wd_seen
        return ((1 if self.place else 0) | (2 if p_only else 0)
                | (4 if p_only and self._betas0 is not None else 0))

    def catch_up_out(self, walks: torch.Tensor, context_radius: int, neg_samples: int,
                     seed: int, noise_offset: int, status: torch.Tensor,
                     noise: Optional[torch.Tensor] = None, step: Optional[int] = None,
                     slot: int = 0) -> None:
        """lazy_out, before pass 1 of the batch ``walks``: the owned out rows its slots
        reference replay their deferred steps up to step - 1 (dw_sgns_owner_out_catch_up).
        ``step``: the Adam step of that batch (default: the current one). ``slot``: the
        workspace and row counts the records are placed with (owner_lazy_steps: 0 / 1 by the
        step's parity)."""
        if not self.lazy_out:
            return
        from shallow_encoders.word2vec.sgns import workspace_for
        step = self.step_count if step is None else int(step)
        n, L = walks.shape
        R, K = int(context_radius), int(neg_samples)
        slots = n * (L - 2 * R) * 2 * R * (1 + K)
        cap = max(1, min(self.S, slots))
        if self._out_rows is None or self._out_rows.numel() < cap:
            self._out_rows = torch.empty(cap, dtype=torch.int32, device=self.device)
        ws = workspace_for(n * (L - 2 * R), 2 * R, K, self.V, self.device, local_rows=self.S,
                           slot=slot)
        counts = self._count_out if slot == 0 else self._count_out2
        self._rows_step = self.rows_major_ok(R, K)
        if not self._rows_step and self._pend_dirty:
            self._flush_out()   # the other form reads the rows as current: settle them first
        flags = (self.out_flags() & 3) | (4 if self._rows_step else 0)
        with torch.cuda.device(self.device):
            _native.call('dw_sgns_owner_out_catch_up', _native.ptr(walks), n, L,
                         int(context_radius), int(neg_samples), self.V, self.d, self.rank,
                         self.world, self.S, _native.ptr(noise), seed & 0xFFFFFFFFFFFFFFFF,
                         int(noise_offset), _native.ptr(self.w_out), _native.ptr(self.m_out),
                         _native.ptr(self.v_out), _native.ptr(self.last_out),
                         _native.ptr(self._claim_out), _native.ptr(counts),
                         _native.ptr(self._out_rows),
                         _native.ptr(self._n_out), _native.ptr(self._hist), step,
                         flags, _native.ptr(status), _native.ptr(ws), ws.numel(),
                         _native.stream(self.device))

    def out_rows_step(self, walks: torch.Tensor, context_radius: int, neg_samples: int,
                      seed: int, noise_offset: int, grad_scale: float, loss_acc: torch.Tensor,
                      status: torch.Tensor, noise: Optional[torch.Tensor] = None,
                      slot: int = 0) -> None:
        """The rows-major out step of the batch ``walks`` (after catch_up_out chose it):
        dw_sgns_owner_out_rows — each touched out row replayed, its records' coefficients and
        loss terms, its gradient and the moments of its Adam step; the rows are left pending
        (p at step - 1 in the table, for the centre pass: sgns_owner_pass1 with
        coefficients_in)."""
        from shallow_encoders.word2vec.sgns import workspace_for
        n, L = walks.shape
        R, K = int(context_radius), int(neg_samples)
        ws = workspace_for(n * (L - 2 * R), 2 * R, K, self.V, self.device, local_rows=self.S,
                           slot=slot)
        counts = self._count_out if slot == 0 else self._count_out2
        self._pend_dirty = True
        with torch.cuda.device(self.device):
            _native.call('dw_sgns_owner_out_rows', _native.ptr(walks), n, L, R, K, self.V,
                         self.d, self.rank, self.world, self.S, _native.ptr(noise),
                         seed & 0xFFFFFFFFFFFFFFFF, int(noise_offset), float(grad_scale),
                         _native.ptr(self.w_in_raw), _native.ptr(self.w_out),
                         _native.ptr(self.g_out), _native.ptr(self.m_out),
                         _native.ptr(self.v_out), _native.ptr(self.last_out),
                         _native.ptr(counts), _native.ptr(self.pend_out),
                         _native.ptr(self._hist), self.step_count,
                         _native.ptr(loss_acc), _native.ptr(status), _native.ptr(ws),
                         ws.numel(), _native.stream(self.device))

    def _alloc_in(self, f32: dict) -> None:
        self.params_in = torch.zeros((1, self.V_pad, self.d), **f32)
        self.grads_in = torch.zeros((self.V_pad, self.d), **f32)
        self.m_in = torch.zeros((self.V_pad, self.d), **f32)
        self.v_in = torch.zeros_like(self.m_in)
        self.grad_shard = None
        self.last_in = torch.zeros(self.V_pad, dtype=torch.int32, device=self.device)
        pin = self.device.type == 'cuda'
        self._hist = torch.zeros((HIST_CAP0, 8), **f32)
        self._hist_host = torch.zeros((HIST_CAP0, 8), dtype=torch.float32, pin_memory=pin)
        self._lr_hist = [0.0]
        self._hist_ready, self._hist_key = 0, None
        self._touched = None
        self._claim_in = None      # one rank, rows-major steps: dw_sgns_owner_touch_claim's marks
        self._n_max = 0
        self._n_touched = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._n_host = torch.zeros(1, dtype=torch.int64, pin_memory=pin)
        self._n_event = None
        self._G = None
        self._ar = None

    # ---- views -------------------------------------------------------------------------------
    @property
    def w_in(self) -> torch.Tensor:
        """The in table with every deferred update applied (flushes)."""
        self.flush()
        return self.params_in[0, :self.V]

    @property
    def w_in_raw(self) -> torch.Tensor:
        """The in table as stored: the rows of the current U are current, others may lag."""
        return self.params_in[0, :self.V]

    def _hip(self) -> bool:
        return self._cuda and self.adam_impl is hip_adam

    # ---- the step ------------------------------------------------------------------------------
    def begin_step(self) -> None:
        """Starts Adam step t and records its scalars for the replays. The rows are written
        HIST_AHEAD steps at a time (one host-to-device copy per block, not per step) for the
        current hyper-parameters; a change of lr (a scheduler) rewrites them from step t."""
        self.step_count += 1
        s = self.step_count
        self._wd_seen = self._wd_seen or self.weight_decay != 0
        if self.lazy_out and tuple(self.betas) != self._betas0:
            self._betas0 = None   # the history's betas differ from step to step from now on
        key = (self.lr, tuple(self.betas), self.eps, self.weight_decay)
        if s > self._hist_ready or key != self._hist_key:
            self._write_hist(s, s + HIST_AHEAD - 1)
        self._lr_hist.append(self.lr)

    def _write_hist(self, lo: int, hi: int) -> None:
        """History rows lo..hi (Adam steps) for the current hyper-parameters."""
        if hi >= self._hist.shape[0]:
            cap = max(2 * self._hist.shape[0], hi + 1)
            h = torch.zeros((cap, 8), dtype=torch.float32, device=self.device)
            h[:self._hist.shape[0]] = self._hist
            hh = torch.zeros((cap, 8), dtype=torch.float32, pin_memory=self._cuda)
            hh[:self._hist_host.shape[0]] = self._hist_host
            self._hist, self._hist_host = h, hh
        rows = np.stack([hist_row(t, self.lr, self.betas, self.eps, self.weight_decay)
                         for t in range(lo, hi + 1)])
        self._hist_host[lo:hi + 1] = torch.from_numpy(rows)
        # row 0: the box header over rows 1..hi (the rows past hi are rewritten before use)
        self._hist_host[0] = torch.from_numpy(hist_header(self._hist_host[:hi + 1].numpy(), hi))
        self._hist[0].copy_(self._hist_host[0], non_blocking=True)
        self._hist[lo:hi + 1].copy_(self._hist_host[lo:hi + 1], non_blocking=True)
        self._hist_ready = hi
        self._hist_key = (self.lr, tuple(self.betas), self.eps, self.weight_decay)

    def reserve_history(self, last_step: int) -> None:
        """The Adam-scalar history written up to ``last_step`` ahead of time (a captured step
        replays begin_step without its host-to-device copies: word2vec/graphed.py)."""
        key = (self.lr, tuple(self.betas), self.eps, self.weight_decay)
        lo = self.step_count + 1
        if key != self._hist_key:
            self._write_hist(lo, max(last_step, lo))
        elif last_step > self._hist_ready:
            self._write_hist(self._hist_ready + 1, last_step)

    def prepare(self, walks: torch.Tensor, context_radius: int, neg_samples: int) -> None:
        """The batch's centre order (for pass 1 with order_ready) and its touched rows U. The
        rows-major step on one rank needs neither the order (its centre pass takes the centres
        in walk order) nor a sorted U: the distinct centres are claimed (dw_sgns_owner_touch_claim,
        a few microseconds where the one-block sort took 30-40 on the step's critical path)."""
        from shallow_encoders.word2vec.sgns import sgns_owner_prepare
        n = walks.shape[0] * (walks.shape[1] - 2 * int(context_radius))
        if self._touched is None or self._touched.numel() < max(n, 1):
            self._touched = torch.empty(max(n, 1), dtype=torch.int32, device=self.device)
        if self._rows_step and not self.multi:
            if self._claim_in is None:
                self._claim_in = torch.zeros(self.V_pad, dtype=torch.int32, device=self.device)
            with torch.cuda.device(self.device):
                _native.call('dw_sgns_owner_touch_claim', _native.ptr(walks), walks.shape[0],
                             walks.shape[1], int(context_radius), self.V,
                             _native.ptr(self._claim_in), self.step_count,
                             _native.ptr(self._touched), _native.ptr(self._n_touched), None,
                             None, 0, _native.stream(self.device))
        else:
            sgns_owner_prepare(walks, context_radius, neg_samples, self.V, self.S,
                               touched=self._touched, n_touched=self._n_touched)
        self._n_max = n
        if self.multi:   # |U| sizes the all-reduce (exchange_touched)
            self._n_host.copy_(self._n_touched, non_blocking=True)
            self._n_event = torch.cuda.Event()
            self._n_event.record(torch.cuda.current_stream(self.device))

    def set_touched(self, rows: torch.Tensor) -> None:
        """CPU protocol (tests): the step's touched rows (distinct centre ids)."""
        self._touched = rows.to(device=self.device, dtype=torch.int64)
        self._n_max = int(rows.numel())

    def _rows(self, g_rows: Optional[torch.Tensor], step: int, all_rows: bool = False) -> None:
        """Replay the listed rows (all rows / the touched ones) up to ``step`` (g = 0), or up to
        step - 1 and then apply ``step`` with g_rows."""
        if self._hip():
            if all_rows:
                hip_rows_adam(self.params_in[0], self.m_in, self.v_in, self.last_in, None, None,
                              self.V_pad, None, self._hist, step)
            else:
                hip_rows_adam(self.params_in[0], self.m_in, self.v_in, self.last_in,
                              self._touched, self._n_touched, self._n_max, g_rows, self._hist,
                              step, grad_by_row=g_rows is self.grads_in)
            return
        rows = torch.arange(self.V_pad, device=self.device) if all_rows else self._touched
        upto = step - 1 if g_rows is not None else step
        last = self.last_in[rows]
        lo = int(last.min()) + 1 if rows.numel() else upto + 1
        for s in range(lo, upto + 1):
            sel = rows[last < s]
            if sel.numel():
                self._cpu_adam_rows(sel, None, s)
        if g_rows is not None and rows.numel():
            self._cpu_adam_rows(rows, g_rows, step)
        self.last_in[rows] = torch.clamp(self.last_in[rows], min=step)

    def _cpu_adam_rows(self, rows: torch.Tensor, g: Optional[torch.Tensor], s: int) -> None:
        p, m, v = self.params_in[0][rows], self.m_in[rows], self.v_in[rows]
        gg = torch.zeros_like(p) if g is None else g.clone()
        self.adam_impl(p.view(-1), gg.view(-1), m.view(-1), v.view(-1), s, self._lr_hist[s],
                       self.betas, self.eps, self.weight_decay, False)
        self.params_in[0][rows] = p
        self.m_in[rows] = m
        self.v_in[rows] = v

    def catch_up(self) -> None:
        """Before pass 1: the touched rows replay their missed steps, up to step - 1."""
        self._rows(None, self.step_count - 1)

    def before_pass1(self, walks: torch.Tensor, context_radius: int, neg_samples: int,
                     seed: int, noise_offset: int, status: torch.Tensor) -> None:
        """prepare + catch_up + catch_up_out (after begin_step). With lazy_out on one rank the
        centre order and in-table catch-up (a one-block sort, then ALU-bound replays) run on
        the side stream beside the out rows' claim and catch-up (bandwidth-bound); the current
        stream waits for both."""
        if self.lazy_out and not self.multi:
            # two branches from one fork: the out rows' claim + catch-up (the longer; enqueued
            # first, so a captured graph launches it first) and the centre order + in-table
            # catch-up
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            fork.record(main)
            self.catch_up_out(walks, context_radius, neg_samples, seed, noise_offset, status)
            with torch.cuda.stream(self._side):
                self._side.wait_event(fork)
                self.prepare(walks, context_radius, neg_samples)
                self.catch_up()
                join = torch.cuda.Event()
                join.record(self._side)
            main.wait_event(join)
            return
        self.prepare(walks, context_radius, neg_samples)
        self.catch_up()
        self.catch_up_out(walks, context_radius, neg_samples, seed, noise_offset, status)

    def exchange_touched(self) -> None:
        """After pass 1: G = g_in[U] (those rows cleared); N > 1: all-reduce(SUM) of G, on a side
        stream behind the output-table phase."""
        n_max = self._n_max
        multi = self.multi
        if self._hip() and not multi:
            # one rank: nothing to exchange — update_touched steps each row straight from its
            # g_in row (dw_adam_rows grad_by_row, which clears it): no gather
            self._G = self.grads_in
            return
        fx = self._exact.get(0) if getattr(self, '_exact', None) is not None else None
        if self._hip() and multi and fx is not None:
            # deterministic, N > 1: the touched rows' integer centre sums (deferred by pass 1),
            # gathered and cleared, all-reduced as int64 on the side stream; update_touched
            # converts them (the same floats on every rank as one rank's conversion)
            if self._G is None or self._G.shape[0] < max(n_max, 1):
                self._G = torch.empty((max(n_max, 1), self.d), dtype=torch.float32,
                                      device=self.device)
            self._n_event.synchronize()
            n = int(self._n_host[0])
            rows = self._touched[:n].long()
            self._G64 = fx.acc.index_select(0, rows)
            fx.acc.index_fill_(0, rows, 0)
            self._G_n = n
            if n > 0:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(self._side):
                    self._side.wait_event(ev)
                    self._ar = dist.all_reduce(self._G64, op=dist.ReduceOp.SUM,
                                               group=self.group, async_op=True)
            return
        if self._hip():
            if self._G is None or self._G.shape[0] < max(n_max, 1):
                self._G = torch.empty((max(n_max, 1), self.d), dtype=torch.float32,
                                      device=self.device)
            with torch.cuda.device(self.device):
                _native.call('dw_rows_gather', _native.ptr(self.grads_in), self.V_pad, self.d,
                             _native.ptr(self._touched), _native.ptr(self._n_touched),
                             int(n_max), _native.ptr(self._G), 1, _native.stream(self.device))
            if multi:
                self._n_event.synchronize()   # the batch's |U| (known since prepare)
                n = int(self._n_host[0])
                if n > 0:
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.device))
                    with torch.cuda.stream(self._side):
                        self._side.wait_event(ev)
                        self._ar = dist.all_reduce(self._G[:n], op=dist.ReduceOp.SUM,
                                                   group=self.group, async_op=True)
            return
        rows = self._touched
        self._G = self.grads_in[rows].clone()
        self.grads_in[rows] = 0.0
        if multi:
            dist.all_reduce(self._G, op=dist.ReduceOp.SUM, group=self.group)

    def update_touched(self) -> None:
        """After pass 2 (which still reads the touched rows): Adam step t on them with G."""
        if self._ar is not None:
            self._ar.wait()            # the current stream waits for the all-reduce
            self._ar = None
        if getattr(self, '_G64', None) is not None:   # deterministic N > 1: convert the sums
            n = self._G_n
            if n > 0:
                self._exact.get(0).convert(acc=self._G64, out=self._G[:n])
            self._G64 = None
        self._rows(self._G, self.step_count)

    def flush(self) -> None:
        """Every row up to the current step (before the table is read as a whole); with
        lazy_out the out slice's deferred steps too."""
        if self.step_count > 0:
            self._rows(None, self.step_count, all_rows=True)
            self._flush_out()

    def _flush_out(self) -> None:
        """lazy_out: every out-slice row up to the current step."""
        if self.lazy_out and self.step_count > 0:
            hip_rows_adam(self.w_out, self.m_out, self.v_out, self.last_out, None, None,
                          self.S, None, self._hist, self.step_count, pending=self.pend_out)
            self._pend_dirty = False

    def out_adam_spec(self) -> Optional[dict]:
        spec = super().out_adam_spec()
        if spec is not None and self.lazy_out:
            spec = {'m': self.m_out, 'v': self.v_out, 'last': self.last_out, 'hist': self._hist,
                    'step': self.step_count, 'flags': self.out_flags(),
                    'counts': self._count_out}
        return spec

    def full_w_out(self) -> torch.Tensor:
        self._flush_out()
        return super().full_w_out()

    def in_state_full(self):
        """(m, v) of the in table (replicated here), every row brought current."""
        self.flush()
        return self.m_in[:self.V].clone(), self.v_in[:self.V].clone()

    def out_state_full(self):
        self._flush_out()
        return super().out_state_full()

    def exchange_in(self, overlap_bytes: Optional[float] = None) -> None:
        raise RuntimeError('OwnerLazyTables steps through owner_lazy_step')

    def sync(self) -> None:
        """Nothing is pending between steps (update_touched waits for the all-reduce)."""


def owner_lazy_steps(tables: OwnerLazyTables, batches, context_radius: int,
                     neg_samples: int, *, seed: int, noise_offsets, grad_scale: float,
                     loss_acc: torch.Tensor, status: torch.Tensor, bind=None,
                     side_first: bool = False) -> int:
    """Consecutive owner_lazy_step calls over ``batches`` (int32 [n, L] walks each, known up
    front: GraphedOwnerStep's unrolled steps), pipelined on one rank with the rows-major out
    step (OwnerLazyTables.pipeline_ok; otherwise the plain sequence). Step k + 1's
    preparation — its out records' claim and placement (dw_sgns_owner_out_catch_up, flags 4),
    its centres' touch claim and the catch-up of the centres step k does not touch — runs on one
    side stream beside step k's out rows, from the moment step k - 1 has finished (the buffers
    alternate by step parity: workspace slot, row counts, touched list), and the main stream
    joins it before step k's centre pass. Only the out rows' step, the centre pass and the in
    rows' update stay on the step's critical path. The results equal the sequential steps':
    each kernel reads and writes
    what it would there (the catch-up of step k + 1 skips the centres of step k, which step k
    updates itself). ``bind(k)``: called before enqueueing anything of step k (graph capture:
    binds step k's dw_step_scalars block). Returns the record count of the steps."""
    R, K = int(context_radius), int(neg_samples)
    batches = list(batches)
    offs = list(noise_offsets)
    n_steps = len(batches)
    if n_steps == 0:
        return 0
    if not tables.pipeline_ok(R, K) or any(b.shape != batches[0].shape for b in batches):
        n = 0
        for k, w in enumerate(batches):
            if bind is not None:
                bind(k)
            n += owner_lazy_step(tables, w, R, K, seed=seed, noise_offset=offs[k],
                                 grad_scale=grad_scale, loss_acc=loss_acc, status=status)
        return n
    from shallow_encoders.word2vec.sgns import sgns_owner_pass1
    t = tables
    dev = t.device
    nw, L = batches[0].shape
    t._pipe_alloc(nw, L, R, K, n_steps)
    s0 = t.step_count + 1
    # every Adam-scalar row the steps read, written before the first side launch (begin_step
    # then copies nothing while a side stream reads the history)
    t.reserve_history(s0 + n_steps - 1)
    if t._pend_dirty and not t._rows_step:
        t._flush_out()
    t._rows_step = True
    main = torch.cuda.current_stream(dev)
    side = t._side   # both preparation chains, one after the other
    p = t._pipe
    ring = p['ctr'][:n_steps]
    ring.zero_()   # every step's touch-claim counters: one memset node, not two per step

    def fork_on(stream, fn, k, fork=None):
        if fork is None:
            fork = torch.cuda.Event()
            fork.record(main)
        if bind is not None:
            bind(k)
        with torch.cuda.stream(stream):
            stream.wait_event(fork)
            fn()
            ev = torch.cuda.Event()
            ev.record(stream)
        return ev

    def ahead(k: int, fork=None):
        """Step k's preparation on the side stream, after ``fork`` (default: everything enqueued
        so far): its touch claim and fresh-row catch-up, then its out-record placement (claim,
        sums, scan, slots)."""
        def chains():   # (the placement first: 0.2817-0.2822 against 0.2781-0.2789 ms)
            t._touch_ahead(batches[k], R, s0 + k, k & 1, ring[k])
            t.catch_up_out(batches[k], R, K, seed, offs[k], status, step=s0 + k, slot=k & 1)
        return fork_on(side, chains, k, fork)

    ready = ahead(0)
    slots = batches[0].shape[0] * (L - 2 * R) * 2 * R * (1 + K)
    # step k + 1's preparation forks at step k's start, beside its out rows, on ONE side stream
    # (the out rows then wait for one side branch and the centre pass follows the out rows with no
    # fork in between): 0.279-0.280 against 0.293-0.296 ms at C3 / 64 with the in-row chain there
    # and the placement on a second stream forked after the out rows (round 5's form, both after
    # the out rows: 0.295-0.301; two streams both at the start: 0.299; one stream after the out
    # rows: 0.300-0.306; the centre pass captured before the forks: 0.324;
    # profiles/r06_pipe_order_ab.txt).
    # The main stream joins step k + 1's preparation before step k's centre pass, not at step
    # k + 1's start: each cross-stream edge costs the main chain ~6 us (a barrier where it waits,
    # a signal where the side forks), and at the step boundary the two had met (10-20 us gaps);
    # 0.2635-0.265 against 0.2672-0.2679 ms (profiles/r06_pipe_order_ab.txt). The preparation
    # ends ~20 us before the out rows do, so the centre pass does not wait for it.
    main.wait_event(ready)
    for k in range(n_steps):
        slot = k & 1
        if bind is not None:
            bind(k)
        t.begin_step()
        w = batches[k]
        fork = torch.cuda.Event()   # step k + 1's preparation depends on what precedes this
        fork.record(main)           # point, but is captured after the out rows (launched first:
        # side_first: step k + 1's preparation enqueued before step k's out rows, so that its
        # in-row catch-up is dispatched first — slower early in a run (0.275 against 0.259 ms
        # at C3 / 64 walks, steps 24-424) and faster once the in rows' lags have grown (0.430
        # against 0.484 ms over steps 16,024-20,024; profiles/r06_pipe_order_ab.txt)
        if side_first and k + 1 < n_steps:
            ready = ahead(k + 1, fork)
            if bind is not None:
                bind(k)
        t.out_rows_step(w, R, K, seed, offs[k], grad_scale, loss_acc, status, slot=slot)
        if k + 1 < n_steps:         # 0.2731-0.2737 against 0.2749-0.2750 ms)
            if not side_first:
                ready = ahead(k + 1, fork)
                if bind is not None:
                    bind(k)
            main.wait_event(ready)
        sgns_owner_pass1(t.w_in_raw, t.w_out, t.grads_in, K, walks=w, context_radius=R,
                         owner=t.rank, n_owners=t.world, vocab_size=t.V, seed=seed,
                         noise_offset=offs[k], grad_scale=grad_scale, status=status,
                         order_ready=True, placed=True, coefficients_in=True,
                         walk_order=True, workspace_slot=slot)
        # the step's in rows with their gradient rows (dw_adam_rows grad_by_row clears them)
        hip_rows_adam(t.params_in[0], t.m_in, t.v_in, t.last_in, p['touched'][slot],
                      ring[k, 0:1], nw * (L - 2 * R), t.grads_in, t._hist,
                      t.step_count, grad_by_row=True)
    return slots * n_steps


def owner_lazy_step(tables: OwnerLazyTables, walks: torch.Tensor, context_radius: int,
                    neg_samples: int, *, seed: int, noise_offset: int, grad_scale: float,
                    loss_acc: torch.Tensor, status: torch.Tensor) -> int:
    """One owner-computes step with the touched-row in-table exchange (every rank passes the
    same global batch). Returns this rank's record count."""
    from shallow_encoders.word2vec.sgns import sgns_owner_pass1, sgns_owner_pass2
    tables.begin_step()
    tables.before_pass1(walks, context_radius, neg_samples, seed, noise_offset, status)
    slots = walks.shape[0] * (walks.shape[1] - 2 * context_radius) * 2 * context_radius * (
        1 + neg_samples)
    if tables.lazy_out and tables._rows_step:
        # rows-major: the out rows' whole step, then the centre gradient from its coefficients
        tables.out_rows_step(walks, context_radius, neg_samples, seed, noise_offset,
                             grad_scale, loss_acc, status)
        sgns_owner_pass1(tables.w_in_raw, tables.w_out, tables.grads_in, neg_samples,
                         walks=walks, context_radius=context_radius, owner=tables.rank,
                         n_owners=tables.world, vocab_size=tables.V, seed=seed,
                         noise_offset=noise_offset, grad_scale=grad_scale, status=status,
                         order_ready=True, placed=True, coefficients_in=True,
                         walk_order=not tables.multi)
        tables.exchange_touched()
        tables.update_touched()
        return slots
    sgns_owner_pass1(tables.w_in_raw, tables.w_out, tables.grads_in, neg_samples, walks=walks,
                     context_radius=context_radius, owner=tables.rank, n_owners=tables.world,
                     vocab_size=tables.V, seed=seed, noise_offset=noise_offset,
                     grad_scale=grad_scale, loss_acc=loss_acc, status=status, order_ready=True,
                     placed=bool(tables.out_flags() & 1))
    tables.exchange_touched()
    spec = tables.out_adam_spec()
    n = sgns_owner_pass2(tables.w_in_raw, tables.w_out, tables.g_out, neg_samples, walks=walks,
                         context_radius=context_radius, out_adam=spec, status=status,
                         read_count=tables.world > 1)
    if n is None:   # one owner keeps every slot (no count readback)
        n = slots
    if spec is None:
        tables.out_step()
    tables.update_touched()
    return n
