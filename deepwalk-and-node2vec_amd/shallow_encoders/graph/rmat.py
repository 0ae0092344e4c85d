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

``rmat_graph(..., device=cuda)`` builds the same graph in HBM:
  * dw_rmat_edges draws the same numpy PCG64 stream on the device;
  * dw_graph_isolated lists the isolated nodes;
  * the host draws their patch targets from the numpy stream advanced past the edge draws;
  * dw_csr_from_edges builds the CSR.
C5 (scale 24) then takes seconds instead of minutes and never materialises the edge list on
the host. Both paths give identical arrays (tests/test_gpu_walks.py).
"""
from typing import Tuple

import numpy as np
import torch

from shallow_encoders.graph.csr import CSRGraph, NodeNames

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
    return CSRGraph.from_arrays(row_ptr, col, None, itos=NodeNames(n, name_width(n)))


def name_width(n: int) -> int:
    return 7 if n <= 10_000_000 else 8


def rmat_graph(scale: int, n_edges: int, seed: int = 0, device=None) -> CSRGraph:
    """The R-MAT graph as a CSR — built on the host (numpy), or in HBM when ``device`` is a
    HIP device (identical arrays)."""
    if device is not None and torch.device(device).type == 'cuda':
        return rmat_graph_device(scale, n_edges, seed, device)
    edges, _ = rmat_edges(scale, n_edges, seed)
    return csr_from_edges(1 << scale, edges)


# ---- device build ------------------------------------------------------------------------------
_PCG_MULT = 0x2360ED051FC65DA44385DF649FCCF645
_M128 = (1 << 128) - 1


def _pcg_jump_table(inc: int):
    """(multiplier, increment) of 2^i PCG64 steps, i < 64 (state -> A * state + C mod 2^128)."""
    a, c, out = _PCG_MULT, inc, []
    for _ in range(64):
        out.append((a, c))
        c = (c * (a + 1)) & _M128
        a = (a * a) & _M128
    return out


def _pcg_advance(state: int, k: int, table) -> int:
    i = 0
    while k:
        if k & 1:
            a, c = table[i]
            state = (a * state + c) & _M128
        k >>= 1
        i += 1
    return state


def _u64_pairs(values) -> np.ndarray:
    return np.array([[v & 0xFFFFFFFFFFFFFFFF, v >> 64] for v in values],
                    dtype=np.uint64).reshape(-1)


def rmat_graph_device(scale: int, n_edges: int, seed: int = 0, device='cuda') -> CSRGraph:
    """rmat_graph built in HBM: same uniforms, same dedupe / patch / CSR order."""
    import ctypes

    from shallow_encoders import _native
    dev = _native.require_device(device)
    a, b, c, _ = RMAT_ABCD
    n = 1 << scale
    rng = np.random.default_rng(seed)
    st = rng.bit_generator.state['state']
    s0, inc = int(st['state']), int(st['inc'])
    table = _pcg_jump_table(inc)
    levels = _u64_pairs(_pcg_advance(s0, level * n_edges, table) for level in range(scale))
    jump = np.array([[x & 0xFFFFFFFFFFFFFFFF, x >> 64, y & 0xFFFFFFFFFFFFFFFF, y >> 64]
                     for x, y in table], dtype=np.uint64).reshape(-1)
    nbytes = ctypes.c_size_t(0)
    _native.call('dw_ingest_workspace_bytes', scale, n_edges + n, n, ctypes.byref(nbytes))
    with torch.cuda.device(dev):
        s = _native.stream(dev)
        ws = torch.empty(int(nbytes.value), dtype=torch.uint8, device=dev)
        lv = torch.from_numpy(levels.view(np.int64)).to(dev)
        jp = torch.from_numpy(jump.view(np.int64)).to(dev)
        edges = torch.empty(n_edges + n, dtype=torch.int64, device=dev)   # + room for patches
        count = torch.zeros(2, dtype=torch.int64, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        _native.call('dw_rmat_edges', scale, n_edges, _native.ptr(lv), _native.ptr(jp),
                     inc & 0xFFFFFFFFFFFFFFFF, inc >> 64, a, a + b, a + b + c,
                     _native.ptr(edges), _native.ptr(count), _native.ptr(ws), ws.numel(), s)
        m = int(count[0])
        iso_dev = torch.empty(n, dtype=torch.int32, device=dev)
        _native.call('dw_graph_isolated', _native.ptr(edges), m, n, _native.ptr(iso_dev),
                     _native.ptr(count[1:]), _native.ptr(status), _native.ptr(ws), ws.numel(), s)
        n_iso = int(count[1])
        if n_iso:
            # the patch targets come from the same numpy stream, past the scale*n_edges draws
            iso = iso_dev[:n_iso].cpu().numpy().astype(np.int64)
            rng.bit_generator.advance(scale * n_edges)
            tgt = rng.integers(0, n - 1, size=n_iso)
            tgt = tgt + (tgt >= iso)
            plo, phi = np.minimum(iso, tgt), np.maximum(iso, tgt)
            _, pfirst = np.unique(plo * n + phi, return_index=True)
            pfirst.sort()
            packed = (iso[pfirst].astype(np.uint64) << np.uint64(32)) | tgt[pfirst].astype(
                np.uint64)
            edges[m:m + len(pfirst)].copy_(torch.from_numpy(packed.view(np.int64)))
            m += len(pfirst)
        del iso_dev
        row_ptr = torch.empty(n + 2, dtype=torch.int64, device=dev)
        col = torch.empty(max(2 * m, 1), dtype=torch.int32, device=dev)
        _native.call('dw_csr_from_edges', _native.ptr(edges), m, n, _native.ptr(row_ptr),
                     _native.ptr(col), _native.ptr(status), _native.ptr(ws), ws.numel(), s)
        _native.check_status(status, 'R-MAT device build')
        del ws, edges
    return CSRGraph.from_device(row_ptr, col[:2 * m], NodeNames(n, name_width(n)))


def rmat_networkx(scale: int, n_edges: int, seed: int = 0):
    """The same graph as a networkx.Graph (small scales only: the reference's own data type)."""
    import networkx as nx
    edges, _ = rmat_edges(scale, n_edges, seed)
    n = 1 << scale
    width = name_width(n)
    g = nx.Graph()
    g.add_edges_from((f'n{u:0{width}d}', f'n{v:0{width}d}') for u, v in edges.tolist())
    return g
