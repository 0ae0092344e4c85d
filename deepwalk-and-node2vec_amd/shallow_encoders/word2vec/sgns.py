"""Fused skip-gram negative-sampling step — host side of dw_sgns_walks / dw_sgns_pairs.

One kernel launch replaces the reference's per-batch chain:
collate windows (torch_dataset.py:293-322) -> noise (sampling.py:7-21) -> SkipGram.forward x2
(model.py:79-91) -> NegativeSamplingLoss (loss.py:14-22) -> autograd embedding backward.
The gradient of ``loss`` (the batch MEAN over B' x 2R terms) is accumulated into dense
(V, d) gradient tables; loss sums and metric counts go to a float64[4] device accumulator
(no host synchronisation).

Two call styles:
  * ``sgns_accumulate(...)``: accumulate into caller-owned gradient buffers (the training loop
    and bench: gradients stay resident, the HIP Adam step consumes and zeroes them);
  * ``SGNSLoss.apply(...)``: an autograd Function returning the loss, for callers that drive
    ``loss.backward()`` themselves (e.g. a Lightning loop).
"""
import math
from typing import Callable, Dict, Optional

import torch

# (T = 2R(1+K) <= 256 and V < 2^31 for the records path; larger falls back to 'atomic')
RECORDS_MAX_ROWS = 256

from shallow_encoders import _native


def loss_terms(acc: torch.Tensor, n_terms: int, neg_samples: int) -> Dict[str, torch.Tensor]:
    """Reference loss dict + metrics from the float64[4] accumulator (device tensors)."""
    m = float(max(n_terms, 1))
    pos = (acc[0] / m).float()
    neg = (acc[1] / m).float()
    out = {
        'loss': pos + neg,
        'positive-loss': pos,
        'negative-loss': neg,
        'recall': (acc[2] / m).float(),
        'precision': (1.0 - acc[3] / (m * max(neg_samples, 1))).float(),
    }
    return out


_WORKSPACES: Dict[torch.device, torch.Tensor] = {}


def _use_records(scatter: str, n_ctx: int, neg_samples: int, vocab_size: int) -> bool:
    return (scatter == 'sorted' and n_ctx * (1 + neg_samples) <= RECORDS_MAX_ROWS
            and vocab_size < 2 ** 31)


def workspace_for(n_centres: int, n_ctx: int, neg_samples: int, vocab_size: int,
                  device: torch.device, local_rows: Optional[int] = None,
                  slot: int = 0) -> torch.Tensor:
    """Device workspace of the atomic-free (records) output-table path, cached per device and
    grown on demand (allocated outside any timed region after the first call). ``local_rows``:
    sized for dw_sgns_owner_pass1 (records keyed by the rank's local out-table rows). ``slot``:
    a second workspace (1) for the pipelined step (owner_lazy_steps: the next batch's records
    are placed while this one's are read)."""
    import ctypes
    nbytes = ctypes.c_size_t(0)
    if local_rows is None:
        _native.call('dw_sgns_workspace_bytes', int(n_centres), int(n_ctx), int(neg_samples),
                     int(vocab_size), ctypes.byref(nbytes))
    else:
        _native.call('dw_sgns_owner_workspace_bytes', int(n_centres), int(n_ctx),
                     int(neg_samples), int(vocab_size), int(local_rows), ctypes.byref(nbytes))
    key = device if slot == 0 else (device, int(slot))
    ws = _WORKSPACES.get(key)
    if ws is None or ws.numel() < nbytes.value:
        _WORKSPACES.pop(key, None)
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=device)
        _WORKSPACES[key] = ws
    return ws


def sgns_accumulate(w_in: torch.Tensor, w_out: torch.Tensor, g_in: torch.Tensor,
                    g_out: torch.Tensor, neg_samples: int, *, walks: Optional[torch.Tensor] = None,
                    context_radius: int = 0, inputs: Optional[torch.Tensor] = None,
                    targets: Optional[torch.Tensor] = None, noise: Optional[torch.Tensor] = None,
                    seed: int = 0, noise_offset: int = 0, grad_scale: Optional[float] = None,
                    loss_acc: Optional[torch.Tensor] = None,
                    status: Optional[torch.Tensor] = None, scatter: str = 'sorted',
                    phase: int = 0, out_adam: Optional[dict] = None) -> torch.Tensor:
    """Launch the fused SGNS kernel(s); returns the float64[4] loss accumulator.

    Either ``walks`` (int32 [n, L]) + ``context_radius``, or ``inputs`` (int64 [B] or [B, 1];
    [B, P] with P > 1 = CBOW, the mean of P input rows) + ``targets`` (int64 [B, C]). ``noise``: int64 [B', C, K] replayed negatives or None (device
    Philox keyed by (seed, noise_offset + centre)). ``grad_scale`` defaults to 1/(B'*C).
    ``scatter``: 'sorted' (records + radix sort + per-row gather, no output-table atomics) or
    'atomic' (float atomics straight into g_out).
    ``phase`` (walks only): 0 = the whole update; 1 = pass 1 (g_in final, loss sums, records);
    2 = the output-table phase (g_out) of the preceding phase-1 call with the same arguments.
    ``out_adam`` (phase 2, records path, one device): ``{'m', 'v', 'flags', 'scalars'}`` — the
    output table's Adam step is fused into the phase (w_out updated in place, g_out left zero;
    ShardedTables.out_adam_spec()).
    """
    dev = w_in.device
    V, d = w_in.shape
    if w_out.shape != (V, d) or g_in.shape != (V, d) or g_out.shape != (V, d):
        raise ValueError('embedding tables and gradients must all be (V, d)')
    for t in (w_in, w_out, g_in, g_out):
        if t.dtype != torch.float32:
            raise TypeError('embedding tables and gradients must be float32')
    if scatter not in ('sorted', 'atomic'):
        raise ValueError('scatter must be "sorted" or "atomic"')
    if loss_acc is None:
        loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    K = int(neg_samples)
    with torch.cuda.device(dev):
        s = _native.stream(dev)
        if walks is not None:
            if walks.dtype != torch.int32 or walks.dim() != 2:
                raise TypeError('walks must be int32 [n_walks, L]')
            n, L = walks.shape
            R = int(context_radius)
            n_centres = n * (L - 2 * R)
            C = 2 * R
            if noise is not None and noise.numel() != n_centres * C * K:
                raise ValueError('noise must have B\' * 2R * K entries')
            scale = 1.0 / max(n_centres * C, 1) if grad_scale is None else grad_scale
            ws = workspace_for(n_centres, C, K, V, dev) \
                if _use_records(scatter, C, K, V) else None
            if out_adam is not None:
                if phase != 2 or ws is None:
                    raise ValueError('out_adam fuses the output-table Adam into phase 2 of the '
                                     'records (sorted) path')
                _native.call('dw_sgns_walks_phase2_adam', _native.ptr(walks), n, L, R, K, V, d,
                             _native.ptr(w_in), _native.ptr(w_out), _native.ptr(g_out),
                             _native.ptr(out_adam['m']), _native.ptr(out_adam['v']),
                             _native.ptr(out_adam['flags']), *out_adam['scalars'],
                             _native.ptr(status), _native.ptr(ws), ws.numel(), s)
                return loss_acc
            _native.call('dw_sgns_walks_phase', int(phase), _native.ptr(walks), n, L, R, K, V, d,
                         _native.ptr(w_in), _native.ptr(w_out), _native.ptr(g_in),
                         _native.ptr(g_out), _native.ptr(noise), seed & 0xFFFFFFFFFFFFFFFF,
                         int(noise_offset), float(scale), _native.ptr(loss_acc),
                         _native.ptr(status), _native.ptr(ws), 0 if ws is None else ws.numel(), s)
        else:
            if inputs is None or targets is None:
                raise ValueError('give walks, or inputs and targets')
            if phase != 0:
                raise ValueError('the two-phase form takes walks')
            B, C = targets.shape
            P = 1 if inputs.dim() == 1 else inputs.shape[1]
            if inputs.numel() != B * P:
                raise ValueError('inputs and targets disagree on the batch size')
            if noise is not None and noise.numel() != B * C * K:
                raise ValueError('noise must have B * C * K entries')
            scale = 1.0 / max(B * C, 1) if grad_scale is None else grad_scale
            if P > 1:
                _native.call('dw_sgns_pooled_pairs', _native.ptr(inputs.contiguous()), P,
                             _native.ptr(targets.contiguous()), B, C, K, V, d, _native.ptr(w_in),
                             _native.ptr(w_out), _native.ptr(g_in), _native.ptr(g_out),
                             _native.ptr(noise), seed & 0xFFFFFFFFFFFFFFFF, int(noise_offset),
                             float(scale), _native.ptr(loss_acc), _native.ptr(status), s)
                return loss_acc
            inputs = inputs.reshape(-1)
            ws = workspace_for(B, C, K, V, dev) if _use_records(scatter, C, K, V) else None
            _native.call('dw_sgns_pairs', _native.ptr(inputs.contiguous()),
                         _native.ptr(targets.contiguous()), B, C, K, V, d, _native.ptr(w_in),
                         _native.ptr(w_out), _native.ptr(g_in), _native.ptr(g_out),
                         _native.ptr(noise), seed & 0xFFFFFFFFFFFFFFFF, int(noise_offset),
                         float(scale), _native.ptr(loss_acc), _native.ptr(status),
                         _native.ptr(ws), 0 if ws is None else ws.numel(), s)
    return loss_acc


def sgns_phase2_pieces(w_in: torch.Tensor, g_out: torch.Tensor, neg_samples: int, *,
                       walks: torch.Tensor, context_radius: int, n_pieces: int,
                       piece_rows: int, on_piece: Optional[Callable[[int], None]] = None,
                       status: Optional[torch.Tensor] = None, scatter: str = 'sorted') -> None:
    """Phase 2 of ``sgns_accumulate(walks=...)`` in output-row pieces (after its phase 1 with the
    same walks): the records sort, then piece by piece the gather of rows [p*piece_rows,
    (p+1)*piece_rows) into g_out, calling ``on_piece(p)`` right after each launch — the caller
    can start exchanging those rows while the next pieces run (ShardedTables.exchange_out_piece).
    Atomic mode: phase 1 already completed g_out; on_piece is called for every piece."""
    dev = w_in.device
    V, d = w_in.shape
    if g_out.shape != (V, d):
        raise ValueError('w_in and g_out must both be (V, d)')
    if walks.dtype != torch.int32 or walks.dim() != 2:
        raise TypeError('walks must be int32 [n_walks, L]')
    if n_pieces * piece_rows < V:
        raise ValueError('the pieces must cover every output row')
    n, L = walks.shape
    R, K = int(context_radius), int(neg_samples)
    C = 2 * R
    if not _use_records(scatter, C, K, V):
        for p in range(n_pieces):
            if on_piece is not None:
                on_piece(p)
        return
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = workspace_for(n * (L - 2 * R), C, K, V, dev)
    with torch.cuda.device(dev):
        for p in range(-1, n_pieces):
            _native.call('dw_sgns_walks_phase2_piece', p, int(n_pieces), int(piece_rows),
                         _native.ptr(walks), n, L, R, K, V, d, _native.ptr(w_in),
                         _native.ptr(g_out), _native.ptr(status), _native.ptr(ws), ws.numel(),
                         _native.stream(dev))
            if p >= 0 and on_piece is not None:
                on_piece(p)


def device_noise(n_centres: int, n_ctx: int, neg_samples: int, vocab_size: int, seed: int,
                 noise_offset: int, device) -> torch.Tensor:
    """int64 [B, C, K]: the negatives the fused kernels draw for ``noise=None`` (same Philox
    keys), materialised — needed when rows must be renormalised before the step (max_norm)."""
    out = torch.empty((n_centres, n_ctx, neg_samples), dtype=torch.int64, device=device)
    with torch.cuda.device(device):
        _native.call('dw_sgns_noise', int(n_centres), int(n_ctx), int(neg_samples),
                     int(vocab_size), seed & 0xFFFFFFFFFFFFFFFF, int(noise_offset),
                     _native.ptr(out), _native.stream(device))
    return out


_RENORM_WS: Dict[torch.device, torch.Tensor] = {}


def renorm_(weight: torch.Tensor, ids: torch.Tensor, max_norm: float,
            status: Optional[torch.Tensor] = None) -> None:
    """nn.Embedding(max_norm) lookup side effect on the device: rows ``ids`` (any shape,
    duplicates allowed) with L2 norm > max_norm are scaled to max_norm / (norm + 1e-7)."""
    import ctypes
    V, d = weight.shape
    ids = ids.reshape(-1).to(weight.device, torch.long).contiguous()
    n = ids.numel()
    if n == 0:
        return
    nbytes = ctypes.c_size_t(0)
    _native.call('dw_embedding_renorm_workspace_bytes', n, V, ctypes.byref(nbytes))
    ws = _RENORM_WS.get(weight.device)
    if ws is None or ws.numel() < nbytes.value:
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=weight.device)
        _RENORM_WS[weight.device] = ws
    st = torch.zeros(1, dtype=torch.int32, device=weight.device) if status is None else status
    with torch.cuda.device(weight.device):
        _native.call('dw_embedding_renorm', _native.ptr(weight.detach()), V, d, _native.ptr(ids),
                     n, float(max_norm), _native.ptr(ws), ws.numel(), _native.ptr(st),
                     _native.stream(weight.device))
    if status is None:
        _native.check_status(st, 'embedding renorm')


def sgns_phase_bytes(n_walks: int, L: int, R: int, K: int, d: int, V: int, scatter: str,
                     fused: bool = False) -> Dict[str, float]:
    """Implementation byte model of each SGNS phase per call of dw_sgns_walks: rows of 4d B,
    12-B records {row u32 | coef f32, centre u32}, one centre-gradient RMW row per centre.
    fused: pass 2 also runs the out table's Adam (p, m, v read + written for every row) instead
    of the g_out read-modify-write."""
    centres = n_walks * (L - 2 * R)
    T = 2 * R * (1 + K)
    n_rec = centres * T
    if scatter != 'sorted':
        return {'pass1': centres * (4 * d * (1 + T) + 8 * d + 8 * d * T) + n_walks * L * 4,
                'sort': 0, 'pass2': 0}
    bits = max(1, math.ceil(math.log2(V)))
    touched = V * (1.0 - math.exp(-n_rec / V))   # expected distinct output rows
    return {'pass1': centres * (4 * d * (1 + T) + 8 * d + 12 * T) + n_walks * L * 4,
            'sort': n_rec * (4 + 24 * math.ceil(bits / 11)),
            'pass2': n_rec * (12 + 4 * d) + (V * d * 24 if fused else touched * 8 * d)}


def phase_timing(enable: bool) -> None:
    """Start (and reset) / stop per-phase HIP-event timing of later SGNS calls (profiling)."""
    _native.call('dw_sgns_timing', 1 if enable else 0)


def phase_ms() -> Dict[str, float]:
    """Mean ms per recorded SGNS call: pass 1, records sort, pass 2 (waits for the last call)."""
    import ctypes
    ms = (ctypes.c_double * 3)()
    n = ctypes.c_int64(0)
    _native.call('dw_sgns_phase_ms', ms, ctypes.byref(n))
    return {'pass1': ms[0], 'sort': ms[1], 'pass2': ms[2], 'calls': int(n.value)}


class SGNSLoss(torch.autograd.Function):
    """loss = NegativeSamplingLoss(SkipGram(in, out), SkipGram(in, noise))['loss'], fused.

    forward(w_in, w_out, walks_or_inputs, targets_or_None, noise_or_None, context_radius,
            neg_samples, seed, noise_offset) -> (loss, positive-loss, negative-loss,
            recall, precision); only ``loss`` carries a gradient.
    """

    @staticmethod
    def forward(ctx, w_in, w_out, src, targets, noise, context_radius, neg_samples, seed,
                noise_offset):
        g_in = torch.zeros_like(w_in)
        g_out = torch.zeros_like(w_out)
        if targets is None:
            acc = sgns_accumulate(w_in.detach(), w_out.detach(), g_in, g_out, neg_samples,
                                  walks=src, context_radius=context_radius, noise=noise,
                                  seed=seed, noise_offset=noise_offset)
            n, L = src.shape
            n_terms = n * (L - 2 * context_radius) * 2 * context_radius
        else:
            acc = sgns_accumulate(w_in.detach(), w_out.detach(), g_in, g_out, neg_samples,
                                  inputs=src, targets=targets, noise=noise, seed=seed,
                                  noise_offset=noise_offset)
            n_terms = targets.numel()
        t = loss_terms(acc, n_terms, neg_samples)
        ctx.save_for_backward(g_in, g_out)
        others = (t['positive-loss'], t['negative-loss'], t['recall'], t['precision'])
        ctx.mark_non_differentiable(*others)
        return (t['loss'],) + others

    @staticmethod
    def backward(ctx, grad_loss, *unused):
        g_in, g_out = ctx.saved_tensors
        if grad_loss is not None:
            go = grad_loss.detach().float().contiguous()
            with torch.cuda.device(g_in.device):
                s = _native.stream(g_in.device)
                _native.call('dw_scale', _native.ptr(g_in), g_in.numel(), 1.0, _native.ptr(go), s)
                _native.call('dw_scale', _native.ptr(g_out), g_out.numel(), 1.0, _native.ptr(go),
                             s)
        return g_in, g_out, None, None, None, None, None, None, None


def sgns_owner_pass1(w_in: torch.Tensor, w_out_local: torch.Tensor, g_in: torch.Tensor,
                     neg_samples: int, *, walks: torch.Tensor, context_radius: int, owner: int,
                     n_owners: int, vocab_size: int, noise: Optional[torch.Tensor] = None,
                     seed: int = 0, noise_offset: int = 0, grad_scale: Optional[float] = None,
                     loss_acc: Optional[torch.Tensor] = None,
                     status: Optional[torch.Tensor] = None,
                     order_ready: bool = False, placed: bool = False,
                     coefficients_in: bool = False,
                     walk_order: bool = False,
                     workspace_slot: int = 0) -> Optional[torch.Tensor]:
    """Pass 1 of the owner-computes step (dw_sgns_owner_pass1, N > 1): over the WHOLE global
    batch ``walks`` (int32 [n, L]), only the output slots whose row o has o % n_owners == owner;
    ``w_out_local`` holds those rows (local row o // n_owners). ``g_in`` ([>= V, d]) receives the
    partial centre-table gradient of the owned slots; returns the float64[4] loss accumulator
    (owned terms only). The records stay in the per-device workspace for sgns_owner_pass2.
    ``order_ready``: sgns_owner_prepare already built the centre order for these walks;
    ``placed``: dw_sgns_owner_out_catch_up placed this batch's records (flags & 1): each goes
    straight into its row's segment. ``coefficients_in`` (with ``placed``): the rows-major step
    (OwnerLazyTables.out_rows_step) already formed the coefficients and left the rows it stepped
    pending, their pre-step values in ``w_out_local`` — only the centre gradient is formed (no
    loss sums: returns None); ``walk_order`` (with it): the centres in walk order, no node order
    built or read. ``workspace_slot``: the workspace the batch's records were placed in
    (workspace_for)."""
    dev = w_in.device
    d = w_in.shape[1]
    local_rows = w_out_local.shape[0]
    if w_out_local.shape[1] != d or g_in.shape[1] != d or g_in.shape[0] < vocab_size \
            or w_in.shape[0] < vocab_size:
        raise ValueError('w_in / g_in must be (>= V, d) and w_out_local (local_rows, d)')
    if local_rows * n_owners < vocab_size:
        raise ValueError('the owners\' local rows do not cover the vocabulary')
    for t in (w_in, w_out_local, g_in):
        if t.dtype != torch.float32:
            raise TypeError('embedding tables and gradients must be float32')
    if walks.dtype != torch.int32 or walks.dim() != 2:
        raise TypeError('walks must be int32 [n_walks, L]')
    n, L = walks.shape
    R, K = int(context_radius), int(neg_samples)
    n_centres = n * (L - 2 * R)
    if noise is not None and noise.numel() != n_centres * 2 * R * K:
        raise ValueError('noise must have B\' * 2R * K entries')
    scale = 1.0 / max(n_centres * 2 * R, 1) if grad_scale is None else grad_scale
    if coefficients_in:
        if not placed:
            raise ValueError('coefficients_in needs the placed records (placed=True)')
        loss_acc = None
    elif walk_order:
        raise ValueError('walk_order is the coefficients_in form\'s')
    elif loss_acc is None:
        loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = workspace_for(n_centres, 2 * R, K, vocab_size, dev, local_rows=local_rows,
                       slot=workspace_slot)
    with torch.cuda.device(dev):
        _native.call('dw_sgns_owner_pass1', _native.ptr(walks), n, L, R, K, int(vocab_size), d,
                     int(owner), int(n_owners), local_rows,
                     (1 if order_ready else 0) | (2 if placed else 0)
                     | (4 if coefficients_in else 0) | (8 if walk_order else 0),
                     _native.ptr(w_in), _native.ptr(w_out_local), _native.ptr(g_in),
                     _native.ptr(noise),
                     seed & 0xFFFFFFFFFFFFFFFF, int(noise_offset), float(scale),
                     _native.ptr(loss_acc), _native.ptr(status), _native.ptr(ws), ws.numel(),
                     _native.stream(dev))
    return loss_acc


def sgns_owner_prepare(walks: torch.Tensor, context_radius: int, neg_samples: int,
                       vocab_size: int, local_rows: int, *,
                       touched: Optional[torch.Tensor] = None,
                       n_touched: Optional[torch.Tensor] = None) -> None:
    """dw_sgns_owner_prepare: the centre order of ``walks`` for sgns_owner_pass1(order_ready=True)
    and, with ``touched`` (int32 [>= n_centres], read as uint32) and ``n_touched`` (int64 [1]),
    the sorted distinct centre nodes and their count, on the device."""
    dev = walks.device
    if walks.dtype != torch.int32 or walks.dim() != 2:
        raise TypeError('walks must be int32 [n_walks, L]')
    n, L = walks.shape
    R, K = int(context_radius), int(neg_samples)
    n_centres = n * (L - 2 * R)
    if touched is not None and (touched.numel() < n_centres or touched.dtype != torch.int32
                                or n_touched is None or n_touched.dtype != torch.int64):
        raise ValueError('touched must be int32 [>= n_centres] with an int64 n_touched')
    ws = workspace_for(n_centres, 2 * R, K, vocab_size, dev, local_rows=local_rows)
    with torch.cuda.device(dev):
        _native.call('dw_sgns_owner_prepare', _native.ptr(walks), n, L, R, K, int(vocab_size),
                     int(local_rows), _native.ptr(touched), _native.ptr(n_touched),
                     _native.ptr(ws), ws.numel(), _native.stream(dev))


def sgns_owner_pass2(w_in: torch.Tensor, w_out_local: torch.Tensor, g_out_local: torch.Tensor,
                     neg_samples: int, *, walks: torch.Tensor, context_radius: int,
                     out_adam: Optional[dict] = None,
                     status: Optional[torch.Tensor] = None,
                     read_count: bool = True) -> Optional[int]:
    """Pass 2 of the owner-computes step (dw_sgns_owner_pass2) after sgns_owner_pass1 with the
    same walks: the records sort and gather over the local slice. ``out_adam`` ({'m', 'v',
    'flags', 'scalars'}, OwnerTables.out_adam_spec()) fuses the slice's Adam step in (w_out_local
    updated, g_out_local left zero); {'m', 'v', 'last', 'hist', 'step'}
    (OwnerLazyTables(lazy_out=True)) the lazy exact form; None accumulates g_out_local. Returns the record count
    (the call synchronises the current stream once to read it); ``read_count=False`` skips
    that synchronisation and sorts the slot bound instead (one owner: every slot is kept, so
    the bound is the count) and returns None."""
    import ctypes
    dev = w_in.device
    d = w_in.shape[1]
    local_rows = w_out_local.shape[0]
    if g_out_local.shape != w_out_local.shape or w_out_local.shape[1] != d:
        raise ValueError('w_out_local and g_out_local must both be (local_rows, d)')
    n, L = walks.shape
    R, K = int(context_radius), int(neg_samples)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=dev)
    ws = workspace_for(n * (L - 2 * R), 2 * R, K, w_in.shape[0], dev, local_rows=local_rows)
    n_rec = ctypes.c_int64(0)
    n_rec_p = ctypes.byref(n_rec) if read_count else None
    if out_adam is not None and 'last' in out_adam:      # OwnerLazyTables(lazy_out=True)
        with torch.cuda.device(dev):
            _native.call('dw_sgns_owner_pass2_lazy', n, L, R, K, local_rows, d, _native.ptr(w_in),
                         _native.ptr(w_out_local), _native.ptr(g_out_local),
                         _native.ptr(out_adam['m']), _native.ptr(out_adam['v']),
                         _native.ptr(out_adam['last']), _native.ptr(out_adam['hist']),
                         int(out_adam['step']), int(out_adam.get('flags', 0)),
                         _native.ptr(out_adam.get('counts')), _native.ptr(status),
                         _native.ptr(ws), ws.numel(),
                         None if out_adam.get('flags', 0) & 1 else n_rec_p,
                         _native.stream(dev))
        return int(n_rec.value) if read_count else None
    if out_adam is not None:
        m, v, flags, sc = (_native.ptr(out_adam['m']), _native.ptr(out_adam['v']),
                           _native.ptr(out_adam['flags']), out_adam['scalars'])
    else:
        m = v = flags = None
        sc = (0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0)
    with torch.cuda.device(dev):
        _native.call('dw_sgns_owner_pass2', n, L, R, K, local_rows, d, _native.ptr(w_in),
                     _native.ptr(w_out_local), _native.ptr(g_out_local), m, v, flags, *sc,
                     _native.ptr(status), _native.ptr(ws), ws.numel(), n_rec_p,
                     _native.stream(dev))
    return int(n_rec.value) if read_count else None
