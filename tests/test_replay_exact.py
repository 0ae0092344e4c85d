"""The replay walker's exact picks without CPython's serial sums (csrc/dw_walk.hip:
uniform_pick_exact, node2vec_pick_exact), restated here in Python floats (IEEE doubles, like
the kernel) and checked against the reference's own arithmetic: random_walk_generator.py:49-52
(sum, normalise), :67 / :113 (random.choices = accumulate + bisect_right over cum[:n-1], CPython
3.10 Lib/random.py), with the node2vec weights of :100-108 (1/p for prev, 1/q for neighbours of
prev, 1 otherwise). The margin rule must never return a pick that differs from the serial
arithmetic; where it declines (-1) the kernel runs the serial replay. Uniforms are drawn at
random and also placed next to the boundaries k/n where the rule has to decline.
"""
import bisect
import itertools
import math
import random

import numpy as np
import pytest


def reference_pick(weights, u):
    """random.choices(range(n), weights=normalised weights)[0] with random() = u."""
    s = sum(weights)
    nw = [w / s for w in weights]
    cum = list(itertools.accumulate(nw))
    total = cum[-1] + 0.0
    return bisect.bisect(cum, u * total, 0, len(cum) - 1)


def margin(n, T):
    return (4.5 * n + 20.0) * 2.0 ** -53 * T


def uniform_pick_exact(u, n):
    T = float(n)
    f = u * T
    M = margin(n, T)
    k = math.floor(f)
    if k > T - 1.0:
        k = T - 1.0
    if k >= 1.0 and abs(k - f) <= M:
        return -1
    if k + 1.0 <= T - 1.0 and abs(k + 1.0 - f) <= M:
        return -1
    return int(k)


def node2vec_pick_exact(classes, u, ip, iq):
    """classes: 0 = other (1), 1 = prev (1/p), 2 = neighbour of prev (1/q); the kernel's
    two-pass rule with the same fp64 evaluation order (rounds of 64 only batch the counts)."""
    n = len(classes)
    A = sum(1 for c in classes if c == 1)
    C = sum(1 for c in classes if c == 2)

    def W(na, nb, nc):
        return float(na) * ip + float(nb) + float(nc) * iq
    T = W(A, n - A - C, C)
    UT = u * T
    M = margin(n, T)
    pa = pc = 0
    d_prev = -UT
    for i, c in enumerate(classes):
        pa += c == 1
        pc += c == 2
        d = W(pa, i + 1 - pa - pc, pc) - UT
        if d > 0.0:
            k = min(i, n - 1)
            if k >= 1 and abs(d_prev) <= M:
                return -1
            if k <= n - 2 and abs(d) <= M:
                return -1
            return k
        d_prev = d
    return -1


SIZES = [1, 2, 3, 5, 7, 10, 64, 65, 100, 333, 1000, 4097, 44848]


@pytest.mark.parametrize('n', SIZES)
def test_uniform_pick_matches_reference(n):
    rng = random.Random(n)
    weights = [1] * n                       # DeepWalk, unweighted: ints, like the reference
    us = [rng.random() for _ in range(400)]
    # next to the boundaries k/n, where the serial rounding decides
    for k in list(range(1, min(n, 40))) + [n // 2, n - 1]:
        if 1 <= k < n:
            for eps in (0.0, 1e-17, -1e-17, 2e-16, -2e-16, 1e-13, -1e-13, 1e-9, -1e-9):
                u = k / n + eps
                if 0.0 <= u < 1.0:
                    us.append(u)
    us += [0.0, 1.0 - 2 ** -53, np.nextafter(1.0, 0.0)]
    declined = 0
    for u in us:
        got = uniform_pick_exact(u, n)
        if got < 0:
            declined += 1
            continue
        assert got == reference_pick(weights, u), (n, u)
    assert declined <= len(us) - 400 + 2       # random uniforms essentially never decline
    assert declined >= (1 if n > 1 else 0)     # u = k/n exactly: the rule must decline


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 0.5), (0.3, 3.0), (1.0, 1.0), (2.0, 0.7),
                                 (0.1, 10.0)])
@pytest.mark.parametrize('n', [1, 2, 3, 9, 64, 130, 1000, 5000])
def test_node2vec_pick_matches_reference(p, q, n):
    rng = random.Random(hash((p, q, n)) & 0xFFFF)
    ip, iq = 1 / p, 1 / q
    for trial in range(30 if n < 2000 else 6):
        classes = [2 if rng.random() < 0.3 else 0 for _ in range(n)]
        classes[rng.randrange(n)] = 1       # prev is a neighbour of v
        weights = []
        for c in classes:                   # random_walk_generator.py:100-108
            w = 1
            if c == 1:
                w *= 1 / p
            elif c == 2:
                w *= 1 / q
            weights.append(w)
        s = sum(weights)
        cum = list(itertools.accumulate(w / s for w in weights))
        us = [rng.random() for _ in range(40)]
        for k in (1, n // 3, n - 1):        # at the boundaries cum[k-1]
            if 1 <= k < n:
                for eps in (0.0, 1e-16, -1e-16, 1e-12, -1e-12):
                    u = min(max(cum[k - 1] / cum[-1] + eps, 0.0), np.nextafter(1.0, 0.0))
                    us.append(u)
        n_declined = 0
        for u in us:
            got = node2vec_pick_exact(classes, u, ip, iq)
            if got < 0:
                n_declined += 1
                continue
            assert got == reference_pick(weights, u), (p, q, n, u)
        assert n_declined <= len(us) - 40 + 1


def node2vec_pick_counted(classes, u, ip, iq, A, C, rb=4):
    """csrc/dw_walk.hip n2v_pick_counted_rb: the class counts A, C of the step are known (the
    per-edge counts), so T is too, and the rounds of 64 are classified from the nearer end only
    (the front when u < 1/2, else the back, prefix counts = totals - suffix counts) until the
    round where D crosses 0; the same D expressions, margin and bracketing test as the full
    classification. Returns (pick or -1, rounds classified)."""
    n = len(classes)
    rounds = (n + 63) // 64

    def W(na, nb, nc):
        return float(na) * ip + float(nb) + float(nc) * iq
    T = W(A, n - A - C, C)
    UT = u * T
    M = margin(n, T)
    if not (T - UT > 0.0):
        return -1, 0

    def counts(r):
        seg = classes[r * 64:(r + 1) * 64]
        return sum(1 for c in seg if c == 1), sum(1 for c in seg if c == 2)

    def resolve(r, na, nc, d_before):
        base = r * 64
        ds = []
        pa, pc = na, nc
        for i in range(base, min(n, base + 64)):
            pa += classes[i] == 1
            pc += classes[i] == 2
            ds.append(W(pa, i + 1 - pa - pc, pc) - UT)
        over = [j for j, d in enumerate(ds) if d > 0.0]
        if not over:
            return -1
        first = over[0]
        k = base + first
        d_k = ds[first]
        d_km1 = ds[first - 1] if first > 0 else d_before
        if k >= 1 and abs(d_km1) <= M:
            return -1
        if k <= n - 2 and abs(d_k) <= M:
            return -1
        return k

    scanned = 0
    if u < 0.5:
        na = nc = 0
        d_prev = -UT
        for r0 in range(0, rounds, rb):
            scanned += rb
            for r in range(r0, min(r0 + rb, rounds)):
                a, c = counts(r)
                end = min((r + 1) * 64, n)
                d_end = W(na + a, end - na - a - nc - c, nc + c) - UT
                if d_end > 0.0:
                    return resolve(r, na, nc, d_prev), scanned
                d_prev, na, nc = d_end, na + a, nc + c
        return -1, scanned
    sa = sc = 0
    for r0 in range(rounds - 1, -1, -rb):
        scanned += rb
        for r in range(r0, max(r0 - rb, -1), -1):
            a, c = counts(r)
            ba, bc = A - sa - a, C - sc - c
            base = r * 64
            d_before = W(ba, base - ba - bc, bc) - UT
            if not (d_before > 0.0):
                return resolve(r, ba, bc, d_before), scanned
            sa, sc = sa + a, sc + c
    return -1, scanned


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0), (2.0, 0.7), (0.1, 10.0)])
@pytest.mark.parametrize('n', [1, 2, 63, 64, 65, 200, 1000, 5000])
def test_node2vec_counted_pick_equals_full_classification(p, q, n):
    """The nearer-end scan with the step's class counts given (the per-edge counts of
    dw_edge_common_counts) returns exactly what the full classification returns — the same
    pick, or the same decline to the serial replay — at random and boundary uniforms, and
    classifies about a quarter of the rounds on average."""
    rng = random.Random(hash((p, q, n, 'cn')) & 0xFFFF)
    ip, iq = 1 / p, 1 / q
    frac = []
    for trial in range(20 if n < 2000 else 5):
        classes = [2 if rng.random() < 0.3 else 0 for _ in range(n)]
        classes[rng.randrange(n)] = 1
        A = sum(1 for c in classes if c == 1)
        C = sum(1 for c in classes if c == 2)
        weights = [1 / p if c == 1 else 1 / q if c == 2 else 1 for c in classes]
        s = sum(weights)
        cum = list(itertools.accumulate(w / s for w in weights))
        us = [rng.random() for _ in range(40)]
        for k in (1, n // 3, n // 2, n - 1):
            if 1 <= k < n:
                for eps in (0.0, 1e-16, -1e-16, 1e-12, -1e-12):
                    us.append(min(max(cum[k - 1] / cum[-1] + eps, 0.0), np.nextafter(1.0, 0.0)))
        for u in us:
            got, scanned = node2vec_pick_counted(classes, u, ip, iq, A, C, rb=1)
            assert got == node2vec_pick_exact(classes, u, ip, iq), (p, q, n, u)
            frac.append(scanned / ((n + 63) // 64))
    if n >= 1000:
        assert np.mean(frac) < 0.35
