"""Synthetic R-MAT power-law graphs (the BASELINE configs C3/C4/C5), built straight to CSR.

Spec (BASELINE.md "Synthetic graph RMAT-20"):
  * quadrant probabilities (a, b, c, d) = (0.57, 0.19, 0.19, 0.05);
  * ``numpy.random.default_rng(seed)``; one uniform per bit per edge, most significant bit
    first: ``r = rng.random(n_edges)`` for each of the ``scale`` levels, then
    ``src |= (r >= a+b)``, ``dst |= (a <= r < a+b) | (r >= a+b+c)`` at that bit;
  * self-loops dropped, undirected duplicates removed (first occurrence kept, edge order =
    order of first draw);
  * every isolated node then gets one edge to ``rng.integers(0, N-1)`` (shifted past itself),
    appended in increasing node order (the reference walker crashes on degree 0 —
    random_walk_generator.py:68 raises IndexError);
  * unweighted; node ``i`` is named ``n%07d`` (``n%08d`` from 10^7 nodes) so that the
    vocabulary's lexicographic order is the numeric one and node i has vocabulary id i+1.

The CSR neighbour order equals what ``nx.Graph().add_edges_from(edges)`` would give (each
row lists its edges in edge-list order), so the reference walker run on the networkx graph
and the device walker run on this CSR see identical neighbour lists.
"""
from typing import Tuple

import numpy as np

from shallow_encoders.graph.csr import CSRGraph

RMAT_ABCD = (0.57, 0.19, 0.19, 0.05)


def rmat_edges(scale: int, n_edges: int, seed: int = 0,
               abcd: Tuple[float, float, float, float] = RMAT_ABCD) -> Tuple[np.ndarray, int]:
    """Undirected R-MAT edge list int64 [E, 2] (deduplicated, isolated nodes patched)."""
    a, b, c, _ = abcd
    n = 1 << scale
    rng = np.random.default_rng(seed)
    src = np.zeros(n_edges, dtype=np.int64)
    dst = np.zeros(n_edges, dtype=np.int64)
    for level in range(scale):
        r = rng.random(n_edges)
        bit = np.int64(1) << np.int64(scale - 1 - level)
        src |= np.where(r >= a + b, bit, 0)
        dst |= np.where(((r >= a) & (r < a + b)) | (r >= a + b + c), bit, 0)
    keep = src != dst
    src, dst = src[keep], dst[keep]
    lo, hi = np.minimum(src, dst), np.maximum(src, dst)
    key = lo * n + hi
    _, first = np.unique(key, return_index=True)
    first.sort()
    edges = np.stack([src[first], dst[first]], axis=1)
    deg = np.bincount(edges.ravel(), minlength=n)
    iso = np.flatnonzero(deg == 0)
    n_patched = len(iso)
    if n_patched:
        tgt = rng.integers(0, n - 1, size=n_patched)
        tgt = tgt + (tgt >= iso)
        patch = np.stack([iso, tgt], axis=1)
        # a patch edge may duplicate another patch edge (u->v and v->u): keep the first
        plo, phi = np.minimum(patch[:, 0], patch[:, 1]), np.maximum(patch[:, 0], patch[:, 1])
        _, pfirst = np.unique(plo * n + phi, return_index=True)
        pfirst.sort()
        edges = np.concatenate([edges, patch[pfirst]], axis=0)
    return edges, n_patched


def csr_from_edges(n: int, edges: np.ndarray) -> CSRGraph:
    """CSR (vocab ids = node + 1) with rows in edge-list order, as networkx would list them."""
    E = len(edges)
    # interleave (u->v, v->u) per edge and stable-sort by source: row order == edge order
    src = np.empty(2 * E, dtype=np.int64)
    dst = np.empty(2 * E, dtype=np.int64)
    src[0::2], dst[0::2] = edges[:, 0], edges[:, 1]
    src[1::2], dst[1::2] = edges[:, 1], edges[:, 0]
    order = np.argsort(src, kind='stable')
    col = (dst[order] + 1).astype(np.int32)
    deg = np.bincount(src, minlength=n)
    row_ptr = np.zeros(n + 2, dtype=np.int64)
    np.cumsum(deg, out=row_ptr[2:])
    width = 7 if n <= 10_000_000 else 8
    itos = ['<unk>'] + [f'n{i:0{width}d}' for i in range(n)]
    return CSRGraph.from_arrays(row_ptr, col, None, itos=itos)


def rmat_graph(scale: int, n_edges: int, seed: int = 0) -> CSRGraph:
    edges, _ = rmat_edges(scale, n_edges, seed)
    return csr_from_edges(1 << scale, edges)


def rmat_networkx(scale: int, n_edges: int, seed: int = 0):
    """The same graph as a networkx.Graph (small scales only: the reference's own data type)."""
    import networkx as nx
    edges, _ = rmat_edges(scale, n_edges, seed)
    n = 1 << scale
    width = 7 if n <= 10_000_000 else 8
    g = nx.Graph()
    g.add_edges_from((f'n{u:0{width}d}', f'n{v:0{width}d}') for u, v in edges.tolist())
    return g
