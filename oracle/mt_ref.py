"""ORACLE — CPython's MT19937 stream and its chained, jump-ahead form (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use this module.

Restates, in numpy, what dw_mt.hip / dw_mt_host.cpp compute, so the CPU suite can pin the
algorithm against CPython's own ``random`` before the device is judged by it:
  * the raw word sequence x[] of MT19937 (Modules/_randommodule.c genrand_uint32's in-place
    twist, as the linear recurrence x[k] = x[k-227] ^ f(x[k-624], x[k-623]));
  * tempering and genrand_res53 (random.random(): ((a >> 5) * 2^26 + (b >> 6)) / 2^53);
  * MT19937's characteristic polynomial phi (135 terms; ``annihilates`` checks it kills the
    sequence's bit planes) and t^J mod phi with Python integers as GF(2) polynomials;
  * the jump x[J + j] = XOR_{l : [t^l] (t^J mod phi) = 1} x[l + j], j >= 1;
  * the chained generation of dw_mt_uniforms (chains of S windows of 624 words; a double whose
    two words straddle a window or a chain).
The reference consumes this stream one value per walk step (random_walk_generator.py:68,113).
"""
from typing import Sequence, Tuple

import numpy as np

N, M = 624, 397
MATRIX_A, UPPER, LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF
DEG = 19937
PHI_TERMS = (  # exponents of phi below t^19937; phi = t^19937 + sum t^e
    0, 1189, 1416, 1585, 1643, 1870, 2493, 2773, 3000, 3227, 3454, 3681, 3908, 4135, 4362, 4753,
    5661, 6337, 6569, 7129, 7477, 7525, 7583, 7752, 7979, 8206, 9505, 9901, 9969, 10128, 10693,
    10761, 10920, 11089, 11147, 11157, 11215, 11321, 11374, 11384, 11485, 11611, 11712, 11717,
    11838, 11881, 11944, 11997, 12277, 12335, 12393, 12504, 12509, 12620, 12673, 12731, 12736,
    12789, 12905, 12958, 12963, 13137, 13185, 13190, 13243, 13301, 13412, 13528, 13533, 13639,
    13697, 13760, 13813, 13866, 14093, 14151, 14209, 14320, 14325, 14436, 14547, 14552, 14605,
    14721, 14774, 14779, 14953, 15001, 15006, 15059, 15117, 15228, 15344, 15349, 15455, 15513,
    15576, 15629, 15682, 15909, 15967, 16025, 16136, 16141, 16252, 16363, 16368, 16421, 16537,
    16590, 16595, 16817, 16822, 16875, 16933, 17044, 17160, 17271, 17329, 17445, 17498, 17725,
    17783, 17841, 17952, 18068, 18179, 18237, 18406, 18633, 18691, 18860, 19087, 19314)
PHI = sum(1 << e for e in PHI_TERMS) | (1 << DEG)


def raw_sequence(mt: Sequence[int], count: int) -> np.ndarray:
    """x[0 .. count) (uint32) with x[0..623] = mt, one 624-word twist block at a time."""
    nb = max(1, -(-count // N))
    x = np.zeros(nb * N, dtype=np.uint32)
    x[:N] = np.asarray(mt, dtype=np.uint32)
    for b in range(1, nb):
        o = x[(b - 1) * N:b * N]
        nw = x[b * N:(b + 1) * N]
        ext = np.concatenate([o, nw[:1]])           # o[kk + 1], with new[0] after o[623]

        def f(a, bb, m):
            y = (a & np.uint32(UPPER)) | (bb & np.uint32(LOWER))
            return m ^ (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(MATRIX_A),
                                                      np.uint32(0)).astype(np.uint32)
        nw[:227] = f(o[:227], o[1:228], o[397:624])
        nw[227:454] = f(o[227:454], o[228:455], nw[0:227])
        nw[454:623] = f(o[454:623], o[455:624], nw[227:396])
        ext[N] = nw[0]
        nw[623] = f(o[623:624], ext[N:N + 1], nw[396:397])[0]
    return x[:count]


def temper(y: np.ndarray) -> np.ndarray:
    y = np.asarray(y, dtype=np.uint32).copy()
    y ^= y >> np.uint32(11)
    y ^= (y << np.uint32(7)) & np.uint32(0x9D2C5680)
    y ^= (y << np.uint32(15)) & np.uint32(0xEFC60000)
    y ^= y >> np.uint32(18)
    return y


def res53(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """genrand_res53 from two raw words (tempered here)."""
    a = (temper(a) >> np.uint32(5)).astype(np.float64)
    b = (temper(b) >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0)


def stream(mt: Sequence[int], index: int, n: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """n values of random.random() from state (mt, index): (doubles, new array, new index)."""
    last = index + 2 * n - 1
    x = raw_sequence(mt, (last // N + 1) * N)
    w = x[index:index + 2 * n]
    out = res53(w[0::2], w[1::2])
    blk = last // N
    return out, x[blk * N:(blk + 1) * N].copy(), last + 1 - blk * N


def annihilates(x: np.ndarray, ks: Sequence[int]) -> bool:
    """phi(t) kills every bit plane of x: XOR_e x[k + e] == 0 over phi's 135 terms, at each k."""
    terms = np.asarray(PHI_TERMS + (DEG,), dtype=np.int64)
    return all(int(np.bitwise_xor.reduce(x[k + terms])) == 0 for k in ks)


def _mulmod(a: int, b: int) -> int:
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if (a >> DEG) & 1:
            a ^= PHI
    return r


def t_pow_mod(e: int) -> int:
    """t^e mod phi as a Python integer (bit l = coefficient of t^l)."""
    r, base = 1, 2
    while e:
        if e & 1:
            r = _mulmod(r, base)
        e >>= 1
        if e:
            base = _mulmod(base, base)
    return r


def exponents(poly: int) -> np.ndarray:
    return np.array([i for i in range(poly.bit_length()) if (poly >> i) & 1], dtype=np.int64)


def jump(x: np.ndarray, ls: np.ndarray, j: np.ndarray) -> np.ndarray:
    """x[J + j] from the exponents ls of t^J mod phi: XOR_l x[l + j]."""
    return np.bitwise_xor.reduce(x[ls[:, None] + j[None, :]], axis=0)


def uniforms_chained(mt: Sequence[int], index: int, n: int, stride: int, positions: np.ndarray,
                     offsets: np.ndarray) -> Tuple[np.ndarray, np.ndarray, int]:
    """dw_mt_uniforms restated: chains of ``stride`` windows, chain c >= 1 seeded by the jump
    table (positions / offsets as dw_mt_jump_table writes them), doubles assigned to the window
    of their second word. Returns (doubles, final array, final index)."""
    out = np.full(n, np.nan)
    if n == 0:
        return out, np.asarray(mt, dtype=np.uint32), index
    first, last = index, index + 2 * n - 1
    n_windows = last // N + 1
    base = raw_sequence(mt, DEG + 625)
    state = None
    for c in range(-(-n_windows // stride)):
        w0, w1 = c * stride, min((c + 1) * stride, n_windows)
        if c == 0:
            win, carry = np.asarray(mt, dtype=np.uint32), np.uint32(0)
        else:
            ls = positions[offsets[c]:offsets[c + 1]].astype(np.int64)
            got = jump(base, ls, np.arange(1, N + 2))
            carry, win = got[0], got[1:]
        prev = None
        for w in range(w0, w1):
            if w > w0:
                win = raw_sequence(win, 2 * N)[N:]
            p0 = N * w
            a2 = p0 + np.arange(N // 2) * 2 + ((p0 - first + 1) & 1)
            keep = (a2 > first) & (a2 <= last)
            a2 = a2[keep]
            o2 = a2 - p0
            x2 = win[o2]
            x1 = np.where(o2 > 0, win[np.maximum(o2 - 1, 0)],
                          carry if w == w0 else (prev[N - 1] if prev is not None else 0))
            out[(a2 - first) >> 1] = res53(x1.astype(np.uint32), x2)
            if w == n_windows - 1:
                state = (win.copy(), last + 1 - p0)
            prev = win
    return out, state[0], state[1]


def torch_randint(mt: Sequence[int], index: int, n: int, high: int) -> Tuple[np.ndarray, np.ndarray, int]:
    """torch.randint(0, high, (n,)) on torch's CPU generator (aten/src/ATen/core/
    DistributionsHelper.h uniform_int_from_to_distribution; the same MT19937 as CPython's), from
    state (mt, index) in CPython's convention — the reference's generate_noise_batch
    (utils/sampling.py:7-21): below a range of 2^28 ONE 32-bit output per value, ``random() %
    range``; from 2^28 (the threshold of torch 2.10, measured in tests/test_host.py) random64() =
    (first output << 32 | second) % range. Returns (int64 values, new array, new index)."""
    if n == 0:
        return np.zeros(0, dtype=np.int64), np.asarray(mt, dtype=np.uint32), index
    w = 1 if high < (1 << 28) else 2
    last = index + w * n - 1
    x = raw_sequence(mt, (last // N + 1) * N)
    t = temper(x[index:index + w * n]).astype(np.uint64)
    if w == 2:
        t = (t[0::2] << np.uint64(32)) | t[1::2]
    vals = (t % np.uint64(high)).astype(np.int64)
    blk = last // N
    return vals, x[blk * N:(blk + 1) * N].copy(), last + 1 - blk * N
