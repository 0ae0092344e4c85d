"""The exact serial node2vec pick in O(C + log n): Python's left-to-right fp64 sums (sum,
accumulate) over a weight sequence that is constant between a few special positions, replayed
run by run (dw_walk.hip ff_run / n2v_pick_serial_runs).

Within one binade [B, 2B) of the running sum S (ulp u), adding the same double y rounds the
same way every time: fl(S + y) = S + d, d = q u (+ u when the remainder r = y - q u exceeds
u / 2; on a tie the even neighbour, constant once S / u is even). So a run of m equal terms
advances in one step per binade. This file restates that rule in Python (the device mirrors it
line for line) and checks it bit for bit against the plain sequential sums on random and
adversarial cases (ties, dyadic and full-mantissa weights, runs crossing many binades, the
first-step uniform case), then the whole pick against the oracle's choices_index."""
import math
import random

import numpy as np
import pytest

from oracle import walk_ref


class Binade:
    """ff_run's constants for one term y in one binade [lo, hi) of S (non-tie, D >= 1): every
    addition there adds D ulps (dw_walk.hip RunBinade)."""
    def __init__(self):
        self.lo, self.hi, self.u, self.iu, self.D = 1.0, 0.0, 0.0, 0.0, 0


def ff_run(S: float, y: float, m: int, x: float = math.inf, bc: Binade = None):
    """m additions of y to S in fp64 round-to-nearest-even. Returns (S_after, j): j = the first
    addition (1-based) after which S > x (S then stops there), or 0 when none. ``bc``: the
    binade cache of the pass (the device keeps one per pass)."""
    bc = Binade() if bc is None else bc
    done = 0
    while done < m:
        if bc.lo <= S < bc.hi:                 # the cached binade: whole rest of the run?
            room = (bc.hi - S) * bc.iu         # exact: integer ulps to the binade's top
            left = m - done
            if left * bc.D <= room:
                Sj = S + (left * bc.D) * bc.u
                if x < Sj:
                    js = 1 if x < S else int((x - S) * bc.iu) // bc.D + 1
                    return S + (js * bc.D) * bc.u, done + js
                return Sj, 0
        if S > 0.0 and y < S:   # (y >= S: the single step below)
            f, e = math.frexp(S)               # S in [2^(e-1), 2^e)
            B2 = math.ldexp(1.0, e)
            u = math.ldexp(1.0, e - 53)
            iu = math.ldexp(1.0, 53 - e)
            q = math.floor(y * iu)
            r = y - q * u
            k = int(S * iu)
            tie = r == 0.5 * u
            if not tie or k % 2 == 0:
                D = q + (1 if (r > 0.5 * u or (tie and q % 2 == 1)) else 0)
                if D == 0:                     # every remaining addition leaves S as it is
                    return S, (done + 1 if S > x else 0)
                if not tie:
                    bc.lo, bc.hi, bc.u, bc.iu, bc.D = 0.5 * B2, B2, u, iu, D
                G = int((B2 - S) * iu)
                jmax = G // D
                if jmax > 0:
                    j = min(jmax, m - done)
                    if x < B2 and x < S + (j * D) * u:   # the crossing is inside the chunk
                        js = 1 if x < S else int((x - S) * iu) // D + 1
                        return S + (js * D) * u, done + js
                    S = S + (j * D) * u
                    done += j
                    continue
        t = S + y                              # one addition, as the hardware does it
        done += 1
        if t == S:                             # a fixed point: the rest add nothing
            return S, 0 if not (t > x) else done
        S = t
        if S > x:
            return S, done
    return S, 0


def seq_sum(S, y, m, x=math.inf):
    for j in range(1, m + 1):
        S = S + y
        if S > x:
            return S, j
    return S, 0


@pytest.mark.parametrize('seed', range(12))
def test_ff_run_equals_sequential_sum(seed):
    rng = random.Random(seed)
    ys = [1.0, 0.25, 4.0, 1 / 3, 0.1, 2 / 3, 1 / 7, 1.0 / 1_000_003, 0.5 + 2 ** -30,
          1 + 2 ** -20, 3 * 2 ** -40, 2 ** -52, 1.5, 1 / 65_537]
    for _ in range(300):
        y = rng.choice(ys) * (rng.choice([1, 1, 1, rng.random() * 3]))
        S = rng.choice([0.0, y, rng.random(), rng.random() * 1e3, 2 ** rng.randint(-20, 20)])
        m = rng.choice([1, 2, 3, 7, 100, 1000, rng.randint(1, 20000)])
        exp = seq_sum(S, y, m)
        assert ff_run(S, y, m) == exp, (S, y, m)
        # a crossing threshold inside the run, at and around the exact partial sums
        S_m = exp[0]
        for x in (S, S_m, (S + S_m) / 2, np.nextafter((S + S_m) / 2, 0.0), S_m * 0.999,
                  rng.uniform(S, S_m)):
            assert ff_run(S, y, m, x) == seq_sum(S, y, m, x), (S, y, m, x)


def test_ff_run_cached_binade_reuse():
    """One cache across many runs of the same term (as a pass uses it), interleaved with other
    additions: the same sums as the plain sequence."""
    rng = random.Random(5)
    for y in (1.0, 1 / 3, 1.0 / 70_001, 0.1, 2 ** -20 * 3):
        bc = Binade()
        S = S2 = 0.0
        for _ in range(400):
            m = rng.choice([1, 2, 5, 40, 300, rng.randint(1, 5000)])
            S, _ = ff_run(S, y, m, math.inf, bc)
            S2, _ = seq_sum(S2, y, m)
            assert S == S2
            z = rng.choice([y * 4, y * 0.25, y * 3, y / 3])
            S, S2 = S + z, S2 + z


def test_ff_run_ties():
    """Terms with few significant bits reach binades where y sits exactly half an ulp off the
    grid: the rounding alternates to the even neighbour."""
    for y in (1.5, 0.75, 3 * 2 ** -30, 5 * 2 ** -45, 2 ** -50 * 3):
        for S in (0.0, 2 ** 52 * y / 3, 2 ** 51 * y, 2 ** 52 * y + y, 1.0, 2 ** 40):
            for m in (1, 5, 64, 3000):
                assert ff_run(S, y, m) == seq_sum(S, y, m), (S, y, m)
                _, hit = seq_sum(S, y, m)
                mid = seq_sum(S, y, m // 2 + 1)[0]
                assert ff_run(S, y, m, mid) == seq_sum(S, y, m, mid)


def seq_pass(specials, n, one, x=math.inf, hi=None):
    """fp64 left-to-right sum of n terms, ``one`` except at the ascending special positions
    (pos, value), run by run. Returns (S, the first index i < hi whose partial sum exceeds x,
    or None); hi defaults to n."""
    hi = n if hi is None else hi
    S, i = 0.0, 0
    bc = Binade()
    for pos, val in list(specials) + [(n, None)]:
        end = min(pos, hi)
        if end > i:                            # the run of ``one`` over [i, end)
            S, j = ff_run(S, one, end - i, x, bc)
            if j:
                return S, i + j - 1
        if pos >= hi or val is None:
            break
        S = S + val
        if S > x:
            return S, pos
        i = pos + 1
    return S, None


def runs_pick_bs(P, pt, n, U, ip, iq):
    """runs_pick with the binade passes (the device's form for lists longer than 48)."""
    P = [int(i) for i in P]
    s, _ = seq_pass_bs(P, pt, ip, iq, n, 1.0)
    n1, np_, nq = 1.0 / s, ip / s, iq / s
    total, _ = seq_pass_bs(P, pt, np_, nq, n, n1)
    total = total + 0.0
    _, hit = seq_pass_bs(P, pt, np_, nq, n, n1, U * total, hi=n - 1)
    return n - 1 if hit is None else hit


def runs_pick(P, pt, n, U, ip, iq):
    """The reference's pick (node2vec_weights + sum + choices) over N(v) whose weights are 1
    except ip at position pt (-1: none) and iq at the ascending positions P, in O(len(P))
    runs."""
    sp = sorted([(int(i), 'q') for i in P] + ([(int(pt), 'p')] if pt >= 0 else []))
    s, _ = seq_pass([(i, ip if c == 'p' else iq) for i, c in sp], n, 1.0)   # sum(w)
    n1, np_, nq = 1.0 / s, ip / s, iq / s                                     # normalized
    norm = [(i, np_ if c == 'p' else nq) for i, c in sp]
    total, _ = seq_pass(norm, n, n1)                                          # accumulate
    total = total + 0.0
    _, hit = seq_pass(norm, n, n1, U * total, hi=n - 1)   # bisect_right(cum, x, 0, n - 1)
    return n - 1 if hit is None else hit


@pytest.mark.parametrize('seed', range(6))
def test_runs_pick_equals_choices(seed):
    rng = np.random.default_rng(seed)
    for _ in range(150):
        n = int(rng.choice([1, 2, 3, 10, 64, 1000, 5000, 70_000]))
        C = int(rng.integers(0, min(n, int(rng.choice([40, 40, 3000]))) + 1))
        P = np.sort(rng.choice(n, C, replace=False)) if C else np.zeros(0, np.int64)
        pt = -1
        if rng.random() < 0.7 and C < n:
            free = np.setdiff1d(np.arange(min(n, 100_000)), P)
            pt = int(rng.choice(free))
        p = float(rng.choice([0.25, 1.0, 4.0, 1 / 3, 0.3, 2.0, 0.7]))
        q = float(rng.choice([0.25, 1.0, 4.0, 3.0, 0.5, 1 / 3]))
        ip, iq = 1 / p, 1 / q
        w = [1] * n
        for i in P:
            w[i] *= iq
        if pt >= 0:
            w[pt] *= ip
        s = sum(w)
        normalized = [x / s for x in w]
        for U in [rng.random(), 0.0, 1 - 2 ** -53] + [float(rng.random()) for _ in range(2)]:
            exp = walk_ref.choices_index(normalized, U)
            assert runs_pick(P, pt, n, U, ip, iq) == exp, (n, C, pt, p, q, U)
            assert runs_pick_bs(P, pt, n, U, ip, iq) == exp, (n, C, pt, p, q, U)
        # uniforms exactly on the cumulative boundaries (where the fast margin declines)
        cum = np.cumsum(np.asarray(normalized, dtype=np.float64))
        for k in rng.integers(0, n, 3):
            U = float(cum[k]) / (float(cum[-1]) + 0.0) if cum[-1] > 0 else 0.5
            U = min(U, 1 - 2 ** -53)
            exp = walk_ref.choices_index(normalized, U)
            assert runs_pick(P, pt, n, U, ip, iq) == exp
            assert runs_pick_bs(P, pt, n, U, ip, iq) == exp


# ---- the closed form per binade with a binary search over the specials (long lists) --------
def _consts(S, vals):
    """Binade constants when every value adds a fixed number of ulps in S's binade: (u, iu,
    KT, [D per value]) or None (S == 0, a value >= the binade's bottom, or a tie)."""
    if S <= 0.0:
        return None
    f, e = math.frexp(S)
    u, iu = math.ldexp(1.0, e - 53), math.ldexp(1.0, 53 - e)
    B = math.ldexp(1.0, e - 1)
    Ds = []
    for y in vals:
        if y >= B:
            return None
        q = math.floor(y * iu)
        r = y - q * u
        if r == 0.5 * u:
            return None
        Ds.append(q + (1 if r > 0.5 * u else 0))
    return u, iu, 2 ** 53, Ds


def seq_pass_bs(P, pt, vp, vq, n, one, x=math.inf, hi=None):
    """seq_pass over (P: ascending 1/q positions, pt: the 1/p position or -1) by binades: inside
    one, k(t) = S / u after the elements [i, t) is k0 + D1 ones + Dq specials — increasing in
    t — so the binade's end and the crossing of x are found by a binary search over P and a
    division in the run of ones before it; the element that leaves the binade is added as it
    is. pt is added singly. Same (S, index) as seq_pass (dw_walk.hip runs_pass_bs)."""
    hi = n if hi is None else hi
    C = len(P)
    S, i, j = 0.0, 0, 0
    p_left = pt >= 0
    while i < hi:
        cs = _consts(S, (one, vq))
        seg_end = pt if (p_left and pt < hi) else hi
        if cs is not None and i < seg_end:
            u, iu, KT, (D1, Dq) = cs
            k0 = int(S * iu)
            XT = int(x * iu) if x < math.ldexp(KT, 0) * u else None   # x inside the binade

            def k_after(jj):      # k after special jj (j <= jj), counting from i
                return k0 + D1 * (P[jj] + 1 - i - (jj + 1 - j)) + Dq * (jj + 1 - j)
            # specials of this segment: P[j .. jc)
            lo_, hi_ = j, C
            while lo_ < hi_:
                mid = (lo_ + hi_) // 2
                if P[mid] < seg_end:
                    lo_ = mid + 1
                else:
                    hi_ = mid
            jc = lo_
            LIM = KT if XT is None else min(KT, XT)   # the first special past LIM stops
            # first special index in [j, jc) with k_after > LIM
            lo_, hi_ = j, jc
            while lo_ < hi_:
                mid = (lo_ + hi_) // 2
                if k_after(mid) > LIM:
                    hi_ = mid
                else:
                    lo_ = mid + 1
            jf = lo_
            t0 = P[jf - 1] + 1 if jf > j else i
            kb = k_after(jf - 1) if jf > j else k0
            run = (P[jf] if jf < jc else seg_end) - t0          # ones before special jf
            # ones of that run that keep k <= LIM
            m = min(run, (LIM - kb) // D1)
            if XT is not None and m < run and kb + D1 * (m + 1) <= KT:
                # the (m+1)-th one crosses x inside the binade
                S = (kb + D1 * (m + 1)) * u
                return S, t0 + m
            if XT is not None and m == run and jf < jc and k_after(jf) <= KT:
                S = k_after(jf) * u                             # special jf crosses x
                return S, P[jf]
            t = t0 + m
            if t > i:                                           # progress inside the binade
                S = (kb + D1 * m) * u
                i, j = t, jf
                continue
        # one element as it is
        if p_left and pt == i:
            val = vp
            p_left = False
        elif j < C and P[j] == i:
            val = vq
            j += 1
        else:
            val = one
        S = S + val
        if S > x:
            return S, i
        i += 1
    return S, None


@pytest.mark.parametrize('seed', range(8))
def test_binade_pass_equals_sequential(seed):
    rng = np.random.default_rng(seed)
    for _ in range(120):
        n = int(rng.choice([1, 2, 5, 64, 1000, 20_000, 200_000]))
        C = int(rng.integers(0, min(n, int(rng.choice([5, 60, 3000]))) + 1))
        P = np.sort(rng.choice(n, C, replace=False)).tolist() if C else []
        pt = -1
        if rng.random() < 0.7 and C < n:
            cand = int(rng.integers(0, n))
            while cand in set(P[:0]) or cand in P:
                cand = int(rng.integers(0, n))
            pt = cand
        one = float(rng.choice([1.0, 1 / n, 1 / (n + 3), 0.1, 1 / 3]))
        vq = one * float(rng.choice([0.25, 4.0, 1 / 3, 3.0, 2.0, 0.7]))
        vp = one * float(rng.choice([4.0, 0.25, 10 / 3, 1.0]))
        sp = sorted([(i, vq) for i in P] + ([(pt, vp)] if pt >= 0 else []))
        S_ref, _ = seq_pass(sp, n, one)
        assert seq_pass_bs(P, pt, vp, vq, n, one) == (S_ref, None)
        for x in [S_ref * float(rng.random()) for _ in range(3)] + [S_ref, S_ref * 0.5]:
            for hi in (n, max(n - 1, 0)):
                assert seq_pass_bs(P, pt, vp, vq, n, one, x, hi) == seq_pass(sp, n, one, x, hi)
