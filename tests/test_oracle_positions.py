"""The Philox position walker's pick, restated in oracle/philox.py (n2v_pick_pos,
fast_walks_positions), against the reference's node2vec law (CPU; the device walker is held to
this restatement bit for bit in tests/test_gpu_walks.py).

  * the pick is the first neighbour whose exact prefix weight exceeds U*T (rational arithmetic),
    wherever U*T is not within fp64 rounding of a prefix;
  * the walks' second-order transitions follow walk_ref.node2vec_transition (the reference rule,
    random_walk_generator.py:94-119, inverted q included) on karate, chi-square.
"""
from fractions import Fraction

import networkx as nx
import numpy as np
import pytest

from oracle import philox as ph
from oracle import walk_ref


def _exact_pick(pt, P, n, U, p, q):
    ip, iq = Fraction(1) / Fraction(p), Fraction(1) / Fraction(q)
    cls = ['o'] * n
    if pt >= 0:
        cls[pt] = 'p'
    for i in P:
        cls[i] = 'q'
    w = [ip if c == 'p' else iq if c == 'q' else Fraction(1) for c in cls]
    T = sum(w)
    x = Fraction(U) * T
    acc = Fraction(0)
    for i, wi in enumerate(w):
        acc += wi
        if acc > x:
            return i, min(abs(acc - x), abs(acc - wi - x)) / T
    return n - 1, Fraction(0)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0), (0.3, 3.0), (2.0, 0.5)])
def test_position_pick_is_first_prefix_above_u_times_total(p, q):
    rng = np.random.default_rng(int(p * 100 + q))
    checked = 0
    for _ in range(3000):
        n = int(rng.integers(1, 300))
        pt = int(rng.integers(-1, n)) if rng.random() < 0.7 else -1
        others = [i for i in range(n) if i != pt]
        C = int(rng.integers(0, len(others) + 1)) if others else 0
        P = sorted(rng.choice(others, size=C, replace=False).tolist()) if C else []
        r0, r1 = (int(x) for x in rng.integers(0, 2 ** 32, size=2))
        U = ph.uniform53(r0, r1)
        got = ph.n2v_pick_pos(P, C, pt, n, U, 1.0 / p, 1.0 / q)
        exp, gap = _exact_pick(pt, P, n, U, p, q)
        if gap > Fraction(1, 10 ** 12):     # away from a prefix by more than fp64 rounding
            assert got == exp, (n, pt, P, U)
            checked += 1
        assert 0 <= got < n
    assert checked > 2900


def test_position_pick_edges():
    """U = 0 picks 0; U just below 1 picks the last neighbour; a single neighbour is always 0."""
    assert ph.n2v_pick_pos([1, 2], 2, 0, 5, 0.0, 4.0, 0.25) == 0
    u_top = ph.uniform53(2 ** 32 - 1, 2 ** 32 - 1)
    assert ph.n2v_pick_pos([1, 2], 2, 0, 5, u_top, 4.0, 0.25) == 4
    assert ph.n2v_pick_pos([3, 4], 2, 0, 5, u_top, 4.0, 0.25) == 4
    assert ph.n2v_pick_pos([], 0, -1, 1, 0.7, 4.0, 0.25) == 0


def test_fast_walks_positions_law_on_karate():
    g = nx.karate_club_graph()
    nodes = sorted(g.nodes())
    row_ptr = [0, 0]
    col = []
    for u in nodes:
        col.extend(x + 1 for x in g.neighbors(u))
        row_ptr.append(len(col))
    ref = walk_ref.CSR(row_ptr, col)
    p, q = 0.3, 3.0
    t, v = 1, 3                        # node 0 -> node 2: hubs with common neighbours
    n = 60_000
    out = ph.fast_walks_positions(row_ptr, col, [t] * n, 3, p, q, seed=11, walk_id0=0)
    sel = out[out[:, 1] == v][:, 2]
    law = walk_ref.node2vec_transition(ref, t, v, p, q)
    xs = sorted(law)
    counts = np.array([(sel == x).sum() for x in xs], dtype=float)
    assert counts.sum() == len(sel) > 3000
    expected = np.array([law[x] for x in xs]) * len(sel)
    from scipy.stats import chi2
    stat = float(((counts - expected) ** 2 / expected).sum())
    assert chi2.sf(stat, len(xs) - 1) > 1e-3
    # the first step is uniform over N(t)
    first = np.bincount(out[:, 1], minlength=len(row_ptr))[ref.neighbors(t)]
    assert chi2.sf(float(((first - n / len(first)) ** 2 / (n / len(first))).sum()),
                   len(first) - 1) > 1e-3
