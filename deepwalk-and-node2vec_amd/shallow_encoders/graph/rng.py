"""The uniform stream of CPython's global ``random`` module, drawn in bulk.

The reference walker consumes exactly one ``random.random()`` per step
(``random.choices(..., k=1)``, random_walk_generator.py:68,113). To reproduce its walks
bit-exactly, the replay kernel is fed the same doubles. Drawing millions of them one Python
call at a time is slow, so the Mersenne-Twister state is moved into a numpy ``RandomState``
(same MT19937 core, same 53-bit ``(a>>5, b>>6)`` double construction), the block is drawn
there, and the advanced state is written back — the global generator ends exactly where
``n`` calls of ``random.random()`` would have left it.
"""
import random

import numpy as np

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
