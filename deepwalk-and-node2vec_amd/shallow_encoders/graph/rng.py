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


# ---- a generator held in HBM across draws (dw_mt_draw) ------------------------------------------
def _torch_state_words(state: torch.Tensor):
    """torch's CPU generator state (torch.get_rng_state(): aten CPUGeneratorImplStateLegacy,
    little-endian: the_initial_seed u64, left i32, seeded i32, next u64, state u64[624], then the
    normal-sample cache) -> (624 uint32 words, index in CPython's convention: the position of the
    next output in the array, 624 = twist first). aten's mt19937 decrements ``left`` per draw and
    twists when it reaches 0, so index = 625 - left (seeding leaves left = 1: twist first)."""
    b = state.numpy()
    left = int(b[8:12].view(np.int32)[0])
    words = b[24:24 + 624 * 8].view(np.uint64).astype(np.uint32)
    return words, 625 - left


def _torch_state_with(state: torch.Tensor, words: np.ndarray, index: int) -> torch.Tensor:
    """``state`` with the twister's array and position replaced (left = 625 - index, next =
    index); the seed and the normal-sample cache untouched."""
    b = state.numpy().copy()
    b[8:12] = np.array([625 - index], dtype=np.int32).view(np.uint8)
    b[16:24] = np.array([index], dtype=np.uint64).view(np.uint8)
    b[24:24 + 624 * 8] = np.asarray(words, dtype=np.uint64).view(np.uint8)
    return torch.from_numpy(b)


class DeviceMT:
    """An MT19937 generator whose state stays in HBM between draws (dw_mt_draw): CPython's
    ``random`` (``uniforms``: random.random(), the walkers' stream, random_walk_generator.py:
    68,113) or torch's CPU generator (``randint``: torch.randint(0, high, ...), the reference's
    negatives, utils/sampling.py:7-21). No host round trip per draw: the host only follows the
    index (a pure function of the draw counts), and the state returns to Python / torch on
    ``to_random`` / ``to_torch``. ``device_index=True`` reads the index on the device instead,
    so launches can be captured once and replayed (word2vec/graphed.py)."""

    def __init__(self, words: np.ndarray, index: int, device, device_index: bool = False):
        from shallow_encoders import _native
        self.device = _native.require_device(device)
        st = np.empty(625, dtype=np.uint32)
        st[:624] = np.asarray(words, dtype=np.uint32)
        st[624] = int(index)
        self.state = torch.from_numpy(st.view(np.int32).copy()).to(self.device)
        self.scratch = torch.empty(625, dtype=torch.int32, device=self.device)
        self.index = None if device_index else int(index)
        self.n_cu = torch.cuda.get_device_properties(self.device).multi_processor_count
        self._ws = None   # this generator's own jump workspace (no sharing across streams)

    @classmethod
    def from_random(cls, device=None, rng: random.Random = None, **kw) -> 'DeviceMT':
        rng = random._inst if rng is None else rng  # noqa: SLF001
        st = np.asarray(rng.getstate()[1], dtype=np.uint32)
        return cls(st[:624], int(st[624]), device, **kw)

    @classmethod
    def from_torch(cls, device=None, **kw) -> 'DeviceMT':
        words, index = _torch_state_words(torch.get_rng_state())
        return cls(words, index, device, **kw)

    def _plan(self, mode: int, n: int):
        """(stride, jump positions, offsets, table chains, workspace) of a draw of n values
        (a device index plans for the largest index, 624)."""
        from shallow_encoders import _native
        wpd = 1 if mode == 1 else 2
        idx = 624 if self.index is None else self.index
        windows = (idx + wpd * n - 1) // 624 + 1 if n > 0 else 1
        per = -(-windows // max(1, CHAINS_PER_CU * self.n_cu))
        stride = max(MIN_CHAIN_WINDOWS, -(-per // 64) * 64)
        chains = -(-windows // stride)
        if chains <= 1:
            return stride, None, None, 1, None
        pos, off, n_tab = mt_jump_table(self.device, stride, chains)
        words = int(_native.load().dw_mt_workspace_words(int(chains)))
        if self._ws is None or self._ws.numel() < words:
            self._ws = torch.empty(words, dtype=torch.int32, device=self.device)
        return stride, pos, off, n_tab, self._ws

    def reserve(self, n: int, high: int = 0) -> None:
        """Build the jump table and workspace a draw of n values needs (uniforms: high = 0;
        randint: its high) ahead of time, e.g. before the draw is captured into a graph."""
        self._plan(0 if not high else (1 if int(high) < (1 << 28) else 2), int(n))

    def _draw(self, mode: int, n: int, out: torch.Tensor, high: int = 0) -> torch.Tensor:
        from shallow_encoders import _native
        n = int(n)
        wpd = 1 if mode == 1 else 2
        stride, pos, off, n_tab, ws = self._plan(mode, n)
        with torch.cuda.device(self.device):
            _native.call('dw_mt_draw', mode, _native.ptr(self.state),
                         -1 if self.index is None else self.index, n, _native.ptr(out),
                         int(high), _native.ptr(self.scratch), stride, _native.ptr(pos),
                         _native.ptr(off), n_tab, _native.ptr(ws), 0 if ws is None else ws.numel(),
                         _native.stream(self.device))
        if self.index is not None and n > 0:
            last = self.index + wpd * n - 1
            self.index = last + 1 - 624 * (last // 624)
        return out

    def uniforms(self, n: int, out: torch.Tensor = None) -> torch.Tensor:
        """float64 [n]: the next n random.random() of this generator."""
        if out is None:
            out = torch.empty(int(n), dtype=torch.float64, device=self.device)
        return self._draw(0, n, out)

    def randint(self, high: int, n: int, out: torch.Tensor = None) -> torch.Tensor:
        """int64 [n]: the next n torch.randint(0, high) values of this generator (0 < high <
        2^32: one output per value below 2^28, two from there, as torch takes them)."""
        if not 0 < int(high) < (1 << 32):
            raise ValueError('randint: high must be in (0, 2^32)')
        if out is None:
            out = torch.empty(int(n), dtype=torch.int64, device=self.device)
        return self._draw(1 if int(high) < (1 << 28) else 2, n, out, high)

    def host_state(self):
        """(624 uint32 words, index): synchronises the current stream."""
        st = self.state.cpu().numpy().view(np.uint32)
        return st[:624].copy(), int(st[624])

    def to_random(self, rng: random.Random = None) -> None:
        """Hand the state back to CPython's generator (default: the global one)."""
        rng = random._inst if rng is None else rng  # noqa: SLF001
        version, _, gauss = rng.getstate()
        words, index = self.host_state()
        rng.setstate((version, tuple(int(w) for w in words) + (index,), gauss))

    def to_torch(self) -> None:
        """Hand the state back to torch's CPU generator."""
        words, index = self.host_state()
        torch.set_rng_state(_torch_state_with(torch.get_rng_state(), words, index))
