"""ORACLE — Philox4x32-10 and the fast-mode sampling rules of libdw_hip (TEST INFRASTRUCTURE).

Bit-for-bit host restatement of deepwalk-and-node2vec_amd/csrc/dw_common.h::philox and of the
counter layouts used by the fast walkers (dw_walk.hip) and the device negative sampler
(dw_sgns.hip), so the device's fast mode can be checked exactly, not only statistically.
The walk LAW these rules sample is the reference's (oracle/walk_ref.py); the stream is ours.
"""
from typing import List, Optional, Sequence

import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF
ALWAYS = 0xFFFFFFFF

TAG_DEEPWALK = 0x44570000
TAG_NODE2VEC = 0x4E320000
TAG_SGNS = 0x53470000
TAG_N2V_POS = 0x4E500000


def philox(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 over numpy uint64 arrays holding 32-bit words."""
    x0, x1, x2, x3 = (np.asarray(v, dtype=np.uint64) & MASK for v in (c0, c1, c2, c3))
    k0 = np.uint64(k0 & MASK)
    k1 = np.uint64(k1 & MASK)
    m0, m1 = np.uint64(M0), np.uint64(M1)
    for _ in range(10):
        p0 = m0 * x0
        p1 = m1 * x2
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        x0, x1, x2, x3 = (hi1 ^ x1 ^ k0), lo1, (hi0 ^ x3 ^ k1), lo0
        k0 = np.uint64((int(k0) + W0) & MASK)
        k1 = np.uint64((int(k1) + W1) & MASK)
    return x0, x1, x2, x3


def bounded32(r, n):
    return (np.asarray(r, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)


def bounded64_int(lo, hi, n: int) -> np.ndarray:
    """floor(r64 * n / 2^64) with r64 = hi:lo, by Python integers (the definition; slow)."""
    lo = np.asarray(lo, dtype=np.uint64).ravel()
    hi = np.asarray(hi, dtype=np.uint64).ravel()
    out = np.empty(lo.shape, dtype=np.int64)
    for i in range(lo.size):
        r = (int(hi[i]) << 32) | int(lo[i])
        out[i] = (r * n) >> 64
    return out


def bounded64(lo, hi, n: int) -> np.ndarray:
    """floor(r64 * n / 2^64) with r64 = hi:lo, n < 2^32, vectorised and exact:
    r64 * n = hi*n*2^32 + lo*n, and with lo*n = A*2^32 + a (a < 2^32) the result is
    floor((hi*n + A) / 2^32) — hi*n + A <= (2^32-1)^2 + 2^32 - 1 < 2^64 never wraps.
    Equal to bounded64_int (tests/test_oracle_golden.py)."""
    if not 0 < n < 2 ** 32:
        raise ValueError('bounded64 needs 0 < n < 2^32')
    lo = np.asarray(lo, dtype=np.uint64).ravel()
    hi = np.asarray(hi, dtype=np.uint64).ravel()
    nn = np.uint64(n)
    s32 = np.uint64(32)
    return ((hi * nn + ((lo * nn) >> s32)) >> s32).astype(np.int64)


def accept_threshold(alpha: float, alpha_max: float) -> int:
    r = alpha / alpha_max
    if r >= 1.0:
        return ALWAYS
    t = float(np.floor(r * 4294967296.0))
    return int(min(max(t, 0.0), 4294967294.0))


def first_order_pick(r0: int, r1: int, a: int, n: int, prob_thr=None, alias=None) -> int:
    i = int(bounded32(r0, n))
    if prob_thr is not None:
        t = int(prob_thr[a + i]) & MASK
        if t != ALWAYS and r1 >= t:
            i = int(alias[a + i])
    return i


def fast_walks(row_ptr, col, starts: Sequence[int], length: int, method: str, p: float, q: float,
               seed: int, walk_id0: int, prob_thr=None, alias=None) -> np.ndarray:
    """The walks dw_walk_fast returns (restatement of dw_walk.hip's fast kernels)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    out = np.full((len(starts), length), -1, dtype=np.int32)
    nsets = {}

    def nset(v):
        s = nsets.get(v)
        if s is None:
            s = set(col[row_ptr[v]:row_ptr[v + 1]].tolist())
            nsets[v] = s
        return s

    if method == 'node2vec':
        ip, iq = 1.0 / p, 1.0 / q
        amax = max(1.0, ip, iq)
        thr_p, thr_q, thr_1 = (accept_threshold(ip, amax), accept_threshold(iq, amax),
                               accept_threshold(1.0, amax))
    lanes = np.arange(64, dtype=np.uint64)
    for w, start in enumerate(starts):
        wid = walk_id0 + w
        c0, c1 = wid & MASK, (wid >> 32) & MASK
        v, prev = int(start), -1
        out[w, 0] = v
        for s in range(1, length):
            a, b = int(row_ptr[v]), int(row_ptr[v + 1])
            n = b - a
            if n <= 0:
                break
            if method in ('deepwalk', 'dfs'):
                r = philox(c0, c1, s << 8, TAG_DEEPWALK, k0, k1)
                nxt = int(col[a + first_order_pick(int(r[0]), int(r[1]), a, n, prob_thr, alias)])
            elif prev < 0:
                r = philox(c0, c1, s << 8, TAG_NODE2VEC, k0, k1)
                nxt = int(col[a + first_order_pick(int(r[0]), int(r[1]), a, n, prob_thr, alias)])
            else:
                nxt = None
                rnd = 0
                while nxt is None:
                    r = philox(np.full(64, c0, np.uint64), np.full(64, c1, np.uint64),
                               (np.uint64(s) << np.uint64(8)) | lanes,
                               np.full(64, TAG_NODE2VEC ^ rnd, np.uint64), k0, k1)
                    for lane in range(64):
                        i = first_order_pick(int(r[0][lane]), int(r[1][lane]), a, n, prob_thr,
                                             alias)
                        x = int(col[a + i])
                        if x == prev:
                            t = thr_p
                        elif x in nset(prev):
                            t = thr_q
                        else:
                            t = thr_1
                        if t == ALWAYS or int(r[2][lane]) < t:
                            nxt = x
                            break
                    rnd += 1
            out[w, s] = nxt
            prev, v = v, nxt
    return out


def n2v_w(na: int, nb: int, nc: int, ip: float, iq: float) -> float:
    """dw_walk.hip n2v_w: the exact prefix weight of na 1/p-, nb 1-, nc 1/q-neighbours, in the
    kernel's fp64 evaluation order (no contraction)."""
    return float(na) * ip + float(nb) + float(nc) * iq


def n2v_pick_pos(P: Sequence[int], C: int, pt: int, n: int, U: float, ip: float,
                 iq: float) -> int:
    """dw_walk.hip n2v_pick_pos<false> (the Philox position walker's pick): with t's position pt
    in N(v) (or -1) and the ascending positions P of the C common neighbours, the first i with
    D_i = W(a_i, i + 1 - a_i - c_i, c_i) - U*T > 0 — a binary search over j of D at P[j], then
    one inside the gap (P[j-1], P[j]]; the same fp64 expressions (Python floats are IEEE
    doubles)."""
    A = 1 if pt >= 0 else 0
    T = n2v_w(A, n - A - C, C, ip, iq)
    UT = U * T

    def D(i: int, c: int) -> float:
        a = 1 if (pt >= 0 and pt <= i) else 0
        return n2v_w(a, (i + 1) - a - c, c, ip, iq) - UT
    lo, hi = 0, C
    while lo < hi:
        mid = (lo + hi) >> 1
        if D(int(P[mid]), mid + 1) > 0.0:
            hi = mid
        else:
            lo = mid + 1
    j = lo
    pj = int(P[j]) if j < C else n - 1
    a = int(P[j - 1]) + 1 if j > 0 else 0
    b = pj
    while a < b:
        mid = (a + b) >> 1
        if D(mid, j) > 0.0:
            b = mid
        else:
            a = mid + 1
    return a


def uniform53(r0: int, r1: int) -> float:
    """U from two Philox words as genrand_res53 splits them: (r0 >> 5) * 2^26 + (r1 >> 6),
    times 2^-53 (exact)."""
    return float(((int(r0) >> 5) << 26) | (int(r1) >> 6)) * 2.0 ** -53


def fast_walks_positions(row_ptr, col, starts: Sequence[int], length: int, p: float, q: float,
                         seed: int, walk_id0: int) -> np.ndarray:
    """The walks dw_walk_fast_positions returns (node2vec, unweighted): counter (walk id lo, hi,
    step << 8, TAG_N2V_POS); step 1 bounded32(r.x, deg) (the reference's unbiased first step,
    random_walk_generator.py:97), later steps n2v_pick_pos with U = uniform53(r.x, r.y) over the
    classes of the reference rule (:100-108: x == prev -> 1/p; x in N(prev) -> 1/q), positions
    found here from the neighbour lists (what the device's per-edge index stores)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    col = np.asarray(col, dtype=np.int64)
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    ip, iq = 1.0 / p, 1.0 / q
    out = np.full((len(starts), length), -1, dtype=np.int32)
    nsets = {}

    def nset(v):
        st = nsets.get(v)
        if st is None:
            st = set(col[row_ptr[v]:row_ptr[v + 1]].tolist())
            nsets[v] = st
        return st
    for w, start in enumerate(starts):
        wid = walk_id0 + w
        c0, c1 = wid & MASK, (wid >> 32) & MASK
        v, prev = int(start), -1
        out[w, 0] = v
        for s in range(1, length):
            a, b = int(row_ptr[v]), int(row_ptr[v + 1])
            n = b - a
            if n <= 0:
                break
            r = philox(c0, c1, s << 8, TAG_N2V_POS, k0, k1)
            if prev < 0:
                k = int(bounded32(int(r[0]), n))
            else:
                nb = col[a:b].tolist()
                pt = nb.index(prev) if prev in nset(v) else -1
                P = [i for i, x in enumerate(nb) if x != prev and x in nset(prev)]
                k = n2v_pick_pos(P, len(P), pt, n, uniform53(int(r[0]), int(r[1])), ip, iq)
            nxt = int(col[a + k])
            out[w, s] = nxt
            prev, v = v, nxt
    return out


def device_noise(seed: int, noise_offset: int, n_centres: int, n_ctx: int, k: int,
                 vocab_size: int) -> np.ndarray:
    """The negatives dw_sgns_* draw when noise == NULL: int64 [B', C, K].

    Centre b's negatives are numbered n = j*K + k (context j, k-th negative); Philox call
    m = n // 2, counter (g lo, g hi, m, TAG_SGNS) with g = noise_offset + b, serves the pair
    n = 2m (words x, y = lo, hi) and n = 2m + 1 (words z, w), each through bounded64 (dw_sgns.hip
    noise_id / k_sgns_g16 / k_noise_fill)."""
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    b = (np.arange(n_centres, dtype=np.uint64) + np.uint64(noise_offset))
    jk = np.arange(n_ctx * k, dtype=np.uint64)
    bb = np.repeat(b, n_ctx * k)
    nn = np.tile(jk, n_centres)
    r = philox(bb & np.uint64(MASK), bb >> np.uint64(32), nn >> np.uint64(1),
               np.full(bb.shape, TAG_SGNS, np.uint64), k0, k1)
    odd = (nn & np.uint64(1)).astype(bool)
    lo = np.where(odd, r[2], r[0])
    hi = np.where(odd, r[3], r[1])
    return bounded64(lo, hi, vocab_size).reshape(n_centres, n_ctx, k)


def philox_torch(c0, c1, c2, c3, k0: int, k1: int):
    """philox() over torch int64 tensors holding 32-bit words (any device; the full-size
    checks run it on the GPU). A 32x32-bit product fits an int64 bit pattern; >> 32 of a
    wrapped (negative) product is masked back to the unsigned high word."""
    m32 = 0xFFFFFFFF
    x0, x1, x2, x3 = (t & m32 for t in (c0, c1, c2, c3))
    k0, k1 = k0 & m32, k1 & m32
    for _ in range(10):
        p0 = x0 * M0
        p1 = x2 * M1
        hi0, lo0 = (p0 >> 32) & m32, p0 & m32
        hi1, lo1 = (p1 >> 32) & m32, p1 & m32
        x0, x1, x2, x3 = (hi1 ^ x1 ^ k0), lo1, (hi0 ^ x3 ^ k1), lo0
        k0 = (k0 + W0) & m32
        k1 = (k1 + W1) & m32
    return x0, x1, x2, x3


def bounded64_torch(lo, hi, n: int):
    """bounded64 over int64 tensors for n < 2^31 (then hi*n + A < 2^63: no signed wrap)."""
    if not 0 < n < 2 ** 31:
        raise ValueError('bounded64_torch needs 0 < n < 2^31')
    return (hi * n + ((lo * n) >> 32)) >> 32


def device_noise_torch(seed: int, noise_offset: int, n_centres: int, n_ctx: int, k: int,
                       vocab_size: int, device=None):
    """device_noise() as an int64 torch tensor [B', C, K] computed on ``device`` (one Philox
    call per pair of negatives, as the kernels draw them). Equal to device_noise
    (tests/test_oracle_golden.py); used where B'·C·K is in the tens of millions."""
    import torch
    k0, k1 = seed & MASK, (seed >> 32) & MASK
    nk = n_ctx * k
    calls = (nk + 1) // 2
    b = torch.arange(n_centres, dtype=torch.int64, device=device) + int(noise_offset)
    bb = b.repeat_interleave(calls)
    mm = torch.arange(calls, dtype=torch.int64, device=device).repeat(n_centres)
    r = philox_torch(bb & MASK, bb >> 32, mm, torch.full_like(bb, TAG_SGNS), k0, k1)
    del bb, mm
    even = bounded64_torch(r[0], r[1], vocab_size).view(n_centres, calls)
    odd = bounded64_torch(r[2], r[3], vocab_size).view(n_centres, calls)
    out = torch.stack([even, odd], dim=2).view(n_centres, 2 * calls)[:, :nk]
    return out.reshape(n_centres, n_ctx, k).contiguous()


def alias_tables(row_ptr, weights: Optional[np.ndarray]):
    """Restatement of dw_graph.hip::k_alias_build (Vose, float64): (prob_thr uint32, alias)."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    nnz = int(row_ptr[-1])
    prob = np.zeros(nnz, dtype=np.uint64)
    alias = np.zeros(nnz, dtype=np.int32)
    for r in range(len(row_ptr) - 1):
        a, b = int(row_ptr[r]), int(row_ptr[r + 1])
        n = b - a
        if n == 0:
            continue
        w = [1.0] * n if weights is None else [float(x) for x in weights[a:b]]
        total = 0.0
        for x in w:
            total += x
        scaled = [x * float(n) / total for x in w]
        small: List[int] = []
        large: List[int] = []
        for i in range(n):
            alias[a + i] = i
            (small if scaled[i] < 1.0 else large).append(i)
        while small and large:
            l_ = small.pop()
            g = large.pop()
            prob[a + l_] = int(min(np.floor(scaled[l_] * 4294967296.0), 4294967295.0))
            alias[a + l_] = g
            scaled[g] = (scaled[g] + scaled[l_]) - 1.0
            (small if scaled[g] < 1.0 else large).append(g)
        for g in large:
            prob[a + g] = ALWAYS
        for l_ in small:
            prob[a + l_] = ALWAYS
    return prob.astype(np.uint32), alias
