"""The uniform stream of CPython's global ``random`` module, drawn in bulk — on the host
(``draw_uniforms``, numpy) or in HBM (``draw_uniforms_device``, dw_mt_uniforms).

The reference walker consumes exactly one ``random.random()`` per step
(``random.choices(..., k=1)``, random_walk_generator.py:68,113). To reproduce its walks
bit-exactly, the replay kernel is fed the same doubles. Drawing millions of them one Python
call at a time is slow, so the Mersenne-Twister state is moved into a numpy ``RandomState``
(same MT19937 core, same 53-bit ``(a>>5, b>>6)`` double construction), the block is drawn
there, and the advanced state is written back — the global generator ends exactly where
``n`` calls of ``random.random()`` would have left it.
"""
import random
import threading

import numpy as np
import torch

_CHUNK = 1 << 24


def draw_uniforms(n: int, rng: random.Random = None) -> np.ndarray:
    """Return the next ``n`` values of ``rng.random()`` (default: the global instance)."""
    rng = random._inst if rng is None else rng  # noqa: SLF001  (the module-level generator)
    n = int(n)
    if n <= 0:
        return np.empty(0, dtype=np.float64)
    if n < 64:
        return np.array([rng.random() for _ in range(n)], dtype=np.float64)
    version, internal, gauss = rng.getstate()
    rs = np.random.RandomState()
    rs.set_state(('MT19937', np.asarray(internal[:624], dtype=np.uint32), int(internal[624]),
                  0, 0.0))
    out = rs.random_sample(n)
    _, key, pos, _, _ = rs.get_state()
    rng.setstate((version, tuple(int(k) for k in key) + (int(pos),), gauss))
    return out


def skip_uniforms(n: int, rng: random.Random = None) -> None:
    """Advance the generator by ``n`` ``random()`` calls without keeping the values."""
    n = int(n)
    while n > 0:
        m = min(n, _CHUNK)
        draw_uniforms(m, rng)
        n -= m


def shuffled_range(n: int, rng: random.Random = None) -> np.ndarray:
    """``x = list(range(n)); rng.shuffle(x)`` as an int64 array, bit for bit, and ``rng`` left
    where that shuffle leaves it (default: the global instance). The loop runs in native code
    (dw_host_shuffle: CPython's MT19937 + ``_randbelow`` + ``shuffle``); ~0.5 s -> ~10 ms for 1M
    nodes."""
    rng = random._inst if rng is None else rng  # noqa: SLF001
    n = int(n)
    if n < 4096 or type(rng) is not random.Random:   # small, or a subclass with its own draws
        x = list(range(n))
        rng.shuffle(x)
        return np.asarray(x, dtype=np.int64)
    from shallow_encoders import _native
    version, internal, gauss = rng.getstate()
    state = np.asarray(internal, dtype=np.uint32)          # 624 words + index
    perm = np.empty(n, dtype=np.int64)
    _native.call('dw_host_shuffle', state.ctypes.data, perm.ctypes.data, n)
    rng.setstate((version, tuple(int(v) for v in state), gauss))
    return perm


# ---- the same stream generated on the device (dw_mt_uniforms) ---------------------------------
_MT_TABLES = {}          # (device, window_stride) -> (positions int16, offsets int64, n_chains)
_MT_WS = {}              # (device, stream) -> int32 workspace of the chains' jump windows
_MT_LOCK = threading.Lock()
MIN_CHAIN_WINDOWS = 256  # below this many 624-word windows per chain, one chain (no jump) wins
CHAINS_PER_CU = 2        # chains the generation spreads over, per compute unit


def mt_window_stride(n: int, index: int, n_cu: int) -> int:
    """Windows per chain for a call of n draws: at least MIN_CHAIN_WINDOWS, else a multiple of
    64 just large enough for CHAINS_PER_CU chains per compute unit (a chain costs one jump, ~10^4
    x 625 LDS reads, then its windows one after another); a batch size that repeats reuses its
    jump table."""
    windows = (index + 2 * n - 1) // 624 + 1 if n > 0 else 1
    per = -(-windows // max(1, CHAINS_PER_CU * n_cu))
    return max(MIN_CHAIN_WINDOWS, -(-per // 64) * 64)


def mt_workspace(device: torch.device, n_chains: int) -> torch.Tensor:
    """Device scratch of dw_mt_uniforms (the chains' jump windows), cached and grown per
    (device, stream): two generations enqueued on different streams (or from different host
    threads on their own streams) never share one, so their jump windows cannot overwrite each
    other. Within one stream the launches are ordered, so reuse is safe."""
    from shallow_encoders import _native
    words = int(_native.load().dw_mt_workspace_words(int(n_chains)))
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    with _MT_LOCK:
        ws = _MT_WS.get(key)
        if ws is None or ws.numel() < words:
            ws = torch.empty(max(words, 1), dtype=torch.int32, device=device)
            _MT_WS[key] = ws
        return ws


def mt_jump_table(device: torch.device, window_stride: int, n_chains: int):
    """Device copy of dw_mt_jump_table(window_stride, >= n_chains), cached and grown by doubling
    (the polynomials depend only on the stride, not on the generator's state)."""
    from shallow_encoders import _native
    key = (device, int(window_stride))
    with _MT_LOCK:
        hit = _MT_TABLES.get(key)
        if hit is not None and hit[2] >= n_chains:
            return hit
        want = max(n_chains, 2 * hit[2] if hit is not None else n_chains)
        off = np.zeros(want + 1, dtype=np.int64)
        pos = np.zeros(want * 19937, dtype=np.uint16)
        _native.call('dw_mt_jump_table', int(window_stride), int(want), off.ctypes.data,
                     pos.ctypes.data, pos.size)
        pos_d = torch.from_numpy(pos[:int(off[-1])].view(np.int16).copy()).to(device)
        off_d = torch.from_numpy(off).to(device)
        _MT_TABLES[key] = (pos_d, off_d, want)
        return _MT_TABLES[key]


def draw_uniforms_device(n: int, device=None, rng: random.Random = None,
                         out: torch.Tensor = None, defer: bool = False):
    """``draw_uniforms`` on the device: float64 [n] in HBM, the next n values of ``rng.random()``
    (default: the global instance) generated by dw_mt_uniforms, and the generator advanced past
    them (2.5 KB each way). ``defer=True`` returns ``(out, commit)``: the caller enqueues its
    consumers first and then calls ``commit()``, which waits for the generator alone (an event
    after the state's copy back) and advances ``rng`` — so a walker launched in between overlaps
    the wait. Otherwise the state is handed back before returning ``out``."""
    from shallow_encoders import _native
    rng = random._inst if rng is None else rng  # noqa: SLF001
    dev = _native.require_device(device)
    n = int(n)
    if out is None:
        out = torch.empty(n, dtype=torch.float64, device=dev)
    elif out.numel() != n or out.dtype != torch.float64 or out.device != dev:
        raise ValueError('out must be float64 [n] on the device')
    if n == 0 or type(rng) is not random.Random:   # a subclass may override random()
        if n:
            out.copy_(torch.from_numpy(np.array([rng.random() for _ in range(n)])))
        return (out, lambda: None) if defer else out
    version, internal, gauss = rng.getstate()
    state = np.asarray(internal, dtype=np.uint32)
    index = int(state[624])
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
    stride = mt_window_stride(n, index, n_cu)
    windows = (index + 2 * n - 1) // 624 + 1
    chains = -(-windows // stride)
    pos = off = ws = None
    n_tab = 1
    if chains > 1:
        pos, off, n_tab = mt_jump_table(dev, stride, chains)
        ws = mt_workspace(dev, chains)
    with torch.cuda.device(dev):
        mt = torch.from_numpy(state[:624].view(np.int32).copy()).to(dev, non_blocking=True)
        st_out = torch.empty(625, dtype=torch.int32, device=dev)
        _native.call('dw_mt_uniforms', _native.ptr(mt), index, n, _native.ptr(out),
                     _native.ptr(st_out), stride, _native.ptr(pos), _native.ptr(off), n_tab,
                     _native.ptr(ws), 0 if ws is None else ws.numel(), _native.stream(dev))
        host = torch.empty(625, dtype=torch.int32, pin_memory=True)
        host.copy_(st_out, non_blocking=True)
        done = torch.cuda.Event()
        done.record(torch.cuda.current_stream(dev))

    def commit():
        done.synchronize()
        new = host.numpy().view(np.uint32)
        rng.setstate((version, tuple(int(v) for v in new), gauss))

    if defer:
        return out, commit
    commit()
    return out
