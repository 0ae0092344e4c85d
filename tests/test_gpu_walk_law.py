"""The Philox fast walkers' transition LAW against the reference's, on R-MAT graphs with hubs.

The fast walkers (rng='philox', bench.py's and sge_sg_rmat20.yaml's walker) are bit-exact against
oracle/philox.py, which is the product's own stream; here their law is checked against the
reference's (random_walk_generator.py:61-72 DeepWalk, :94-119 Node2Vec with its inverted q
rule, restated by oracle/walk_ref.node2vec_transition and pinned by the reference's fixtures).

  * node2vec, second-order step P(x | t, v): walks of length 3 start at t; the walks whose
    first step is v give samples of x. Pairs per graph: hub t -> hub v, hub t -> low-degree v,
    low-degree t -> hub v, mid t -> mid v (with common neighbours). (p, q) = (.25, 4) (C5's
    walk) and (1, 1) (C2's). Outcomes are binned by the law's own structure — x == t, x a
    common neighbour of t and v, x another neighbour — each category cut into up to 8 bins of
    consecutive ids, and a chi-square test is run on the bins.
  * node2vec first step (prev = None) and DeepWalk: uniform over N(v); chi-square over every
    neighbour of a hub (R-MAT 12 / 16, and C3's 44,848-neighbour hub for DeepWalk).

Two node2vec walkers: the default over the per-edge position index (one Philox uniform against
the exact prefix weights) and the ballot-rejection walker (layout 'hash' / 'csr'). For the
latter the lane-group size (16 / 8 / 4 lanes per walker, picked from the batch size) and the
layout (edge-inline + adjacency hash vs plain CSR + sorted search) do not change a walk (walks
are pure functions of the walk id): each test asserts that on the first walks of its batch, so
the law shown for one holds for all of them.

Significance: family-wise alpha = 1e-3 with a Bonferroni correction over the N_TESTS tests of
this module: each test passes when its p-value > 1e-3 / N_TESTS. Seeds are fixed, so the
p-values are deterministic.
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import walk_ref

pytestmark = pytest.mark.gpu

PQ = [(0.25, 4.0), (1.0, 1.0)]
PAIR_KINDS = ['hub-hub', 'hub-low', 'low-hub', 'mid-mid']
GRAPHS = ['rmat12', 'rmat16']
DW_GRAPHS = ['rmat12', 'rmat16', 'rmat20']
WALKERS = ['positions', 'rejection']
N_TESTS = len(PQ) * len(GRAPHS) * (len(WALKERS) * len(PAIR_KINDS) + 1) + len(DW_GRAPHS)
ALPHA = 1e-3 / N_TESTS
TARGET = 4000          # samples of x per (t, v) pair
MAX_WALKS = 40_000_000

_CACHE = {}


def _graph(name):
    if name not in _CACHE:
        from shallow_encoders.graph.csr import CSRGraph
        from shallow_encoders.graph.rmat import rmat_graph
        if name == 'rmat12':
            f = golden('walks_rmat12_node2vec_p0.25_q4.npz')
            csr = CSRGraph.from_arrays(f['row_ptr'], f['col'], None)
        elif name == 'rmat16':     # built on the device (== the host build, test_gpu_walks.py)
            csr = rmat_graph(16, 600_000, 0, device=torch.device('cuda', 0))
        else:
            csr = rmat_graph(20, 10_000_000, 0, device=torch.device('cuda', 0))
        ref = walk_ref.CSR(csr.row_ptr, csr.host_col()) if name != 'rmat20' else None
        _CACHE[name] = (csr, ref)
    return _CACHE[name]


def _pair(csr, kind):
    rp = np.asarray(csr.row_ptr)
    col = np.asarray(csr.host_col())
    deg = np.diff(rp)
    nb = lambda u: col[rp[u]:rp[u + 1]]  # noqa: E731
    order = np.argsort(-deg, kind='stable')
    hub = int(order[0])
    if kind == 'hub-hub':
        n = nb(hub)
        return hub, int(n[np.argmax(deg[n])])
    if kind == 'hub-low':
        n = nb(hub)
        cand = n[(deg[n] >= 3) & (deg[n] <= 8)]
        return hub, int(cand[0])
    if kind == 'low-hub':
        v = int(order[1])
        n = nb(v)
        cand = n[(deg[n] >= 2) & (deg[n] <= 8)]
        return int(cand[0]), v
    # mid-mid: degrees in [20, 60] with the most common neighbours
    mids = np.flatnonzero((deg >= 20) & (deg <= 60))
    best, best_c = None, -1
    for t in mids[:400]:
        nt = set(nb(t).tolist())
        for v in nb(t):
            if 20 <= deg[v] <= 60:
                c = len(nt & set(nb(v).tolist()))
                if c > best_c:
                    best, best_c = (int(t), int(v)), c
    return best


def _chi2_p(counts, expected):
    from scipy.stats import chi2
    counts, expected = np.asarray(counts, float), np.asarray(expected, float)
    stat = float(((counts - expected) ** 2 / expected).sum())
    return float(chi2.sf(stat, len(counts) - 1)), stat


def _same_across_lanes_and_layouts(make, starts, big, layout):
    """The walks of the first starts are the same in a small batch (the rejection walker: 16
    lanes per walker) as in the big one (4 lanes), and the rejection walker's are the same with
    the plain-CSR layout."""
    n = min(4096, len(starts))
    small = make(layout).walk_batch(starts[:n], walk_id0=0)
    assert torch.equal(small, big[:n])
    if layout == 'hash':
        plain = make('csr').walk_batch(starts[:n], walk_id0=0)
        assert torch.equal(plain, big[:n])


def _bins(law, t, v, ref, n_samples):
    """Bins of x by the law's structure: [t], common neighbours, others, each category cut
    into up to 8 runs of consecutive ids with >= 5 expected samples per bin."""
    nt = ref.neighbor_set(t)
    cats = {'ret': [], 'common': [], 'other': []}
    for x in sorted(law):
        cats['ret' if x == t else 'common' if x in nt else 'other'].append(x)
    bins = []
    for members in cats.values():
        if not members:
            continue
        pc = sum(law[x] for x in members)
        k = int(max(1, min(8, len(members), math.floor(pc * n_samples / 5))))
        for chunk in np.array_split(np.array(members), k):
            bins.append(chunk)
    return bins


@pytest.mark.parametrize('walker', WALKERS)
@pytest.mark.parametrize('graph', GRAPHS)
@pytest.mark.parametrize('kind', PAIR_KINDS)
@pytest.mark.parametrize('p,q', PQ)
def test_node2vec_second_order_law_vs_reference(graph, kind, p, q, walker, hip_device):
    """walker: 'positions' (the default layout on unweighted graphs: dw_walk_fast_positions,
    one Philox uniform against the prefix weights over the position index) or 'rejection'
    (layout 'hash' / 'csr': the ballot-rejection walker)."""
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    csr, ref = _graph(graph)
    layout = 'indexed' if walker == 'positions' else 'hash'
    t, v = _pair(csr, kind)
    deg_t, deg_v = len(ref.neighbors(t)), len(ref.neighbors(v))
    n = min(MAX_WALKS, TARGET * deg_t)
    starts = torch.full((n,), t, dtype=torch.int32, device=hip_device)

    def make(layout):
        return Node2Vec(csr, 3, p=p, q=q, rng='philox', seed=2024, layout=layout,
                        device=hip_device)
    out = make(layout).walk_batch(starts, walk_id0=0)
    if walker == 'positions':
        assert csr.device_tensors(hip_device).get('n2v_rec') is not None
    _same_across_lanes_and_layouts(make, starts, out, layout)
    x = out[out[:, 1] == v][:, 2].cpu().numpy()
    law = walk_ref.node2vec_transition(ref, t, v, p, q)
    assert set(np.unique(x).tolist()) <= set(law), 'a step left N(v)'
    bins = _bins(law, t, v, ref, len(x))
    counts = [np.isin(x, b).sum() for b in bins]
    expected = [sum(law[int(y)] for y in b) * len(x) for b in bins]
    pv, stat = _chi2_p(counts, expected)
    print(f'{graph} {kind} (t={t}, deg {deg_t}; v={v}, deg {deg_v}) p={p} q={q}: '
          f'{len(x)} samples, {len(bins)} bins, chi2 {stat:.1f}, p-value {pv:.3g}')
    assert len(x) >= 0.5 * TARGET * min(1.0, MAX_WALKS / (TARGET * deg_t))
    assert pv > ALPHA, f'p-value {pv:.3g} <= {ALPHA:.2g}'


@pytest.mark.parametrize('graph', GRAPHS)
@pytest.mark.parametrize('p,q', PQ)
def test_node2vec_first_step_uniform_on_hub(graph, p, q, hip_device):
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    csr, ref = _graph(graph)
    hub = int(np.argmax(np.diff(csr.row_ptr)))
    nbrs = np.array(ref.neighbors(hub))
    n = 30 * len(nbrs)
    starts = torch.full((n,), hub, dtype=torch.int32, device=hip_device)
    out = Node2Vec(csr, 2, p=p, q=q, rng='philox', seed=7, device=hip_device).walk_batch(
        starts, walk_id0=0)
    x = out[:, 1].cpu().numpy()
    counts = np.bincount(np.searchsorted(np.sort(nbrs), x), minlength=len(nbrs))
    assert counts.sum() == n
    pv, stat = _chi2_p(counts, np.full(len(nbrs), n / len(nbrs)))
    print(f'{graph} node2vec first step from hub {hub} (deg {len(nbrs)}): p-value {pv:.3g}')
    assert pv > ALPHA


@pytest.mark.parametrize('graph', DW_GRAPHS)
def test_deepwalk_uniform_law_on_hub(graph, hip_device):
    from shallow_encoders.graph.random_walk_generator import DeepWalk
    csr, _ = _graph(graph)
    rp = np.asarray(csr.row_ptr)
    hub = int(np.argmax(np.diff(rp)))
    nbrs = np.sort(np.asarray(csr.host_col())[rp[hub]:rp[hub + 1]])
    n = 30 * len(nbrs)
    starts = torch.full((n,), hub, dtype=torch.int32, device=hip_device)
    big = DeepWalk(csr, 2, rng='philox', seed=9, device=hip_device).walk_batch(starts,
                                                                                walk_id0=0)
    plain = DeepWalk(csr, 2, rng='philox', seed=9, layout='csr',
                     device=hip_device).walk_batch(starts[:4096], walk_id0=0)
    assert torch.equal(plain, big[:4096])
    x = big[:, 1].cpu().numpy()
    idx = np.searchsorted(nbrs, x)
    assert (nbrs[np.minimum(idx, len(nbrs) - 1)] == x).all(), 'a step left N(hub)'
    counts = np.bincount(idx, minlength=len(nbrs))
    pv, stat = _chi2_p(counts, np.full(len(nbrs), n / len(nbrs)))
    print(f'{graph} DeepWalk from hub {hub} (deg {len(nbrs)}): {n} walks, p-value {pv:.3g}')
    assert pv > ALPHA
