"""Random walk generators — the reference API (random_walk_generator.py:11-151) on gfx950 kernels.

Two sampling modes, one kernel family each (include/dw_hip.h):

* ``rng='python'`` (default, reference-exact): every step consumes ONE double of CPython's
  global ``random`` stream, exactly as ``random.choices(..., k=1)`` does in the reference
  (random_walk_generator.py:68,113). The doubles are generated in HBM from the generator's
  state (rng.draw_uniforms_device: CPython's MT19937 on the device, dw_mt_uniforms; the state is
  handed back so ``random`` continues exactly) and the replay kernel ``dw_walk_replay``
  reproduces CPython's fp64 arithmetic, so ``random.seed(s)`` yields the reference's walks bit
  for bit.
* ``rng='philox'``: ``dw_walk_fast_indexed`` (DeepWalk over the edge-inline CSR, node2vec
  adjacency tests in a per-row hash; the default) or ``dw_walk_fast`` (plain CSR,
  ``layout='csr'``), Philox4x32-10
  keyed by (seed, global walk id); the walk law is the reference's (including its inverted
  node2vec q rule), the stream is not.

``walk(node) -> str`` keeps the reference signature; ``walk_batch`` is the batched device API
(int32 vocabulary ids, shape [n_walks, length]) that feeds the fused SGNS kernel.
"""
import os
import sys
from abc import ABC
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from shallow_encoders import _native
from shallow_encoders.graph.csr import CSRGraph
from shallow_encoders.graph.rng import draw_uniforms_device

_CSR_CACHE_ATTR = '_dw_csr_cache'


def _edge_cn_enabled() -> bool:
    """The node2vec replay's per-edge class counts (dw_edge_common_counts, built once per graph):
    on by default; DW_N2V_EDGE_CN=0 classifies every step's whole N(v) (the same walks)."""
    return os.environ.get('DW_N2V_EDGE_CN', '1') != '0'


def _n2v_index_enabled() -> bool:
    """The node2vec replay over the per-edge position index (dw_n2v_edge_index_build, built once
    per graph within CSRGraph.N2V_INDEX_BYTES; one lane per walker, dw_walk_replay_positions):
    on by default; DW_N2V_POS=0 keeps the wave walker with the counts (the same walks)."""
    return _edge_cn_enabled() and os.environ.get('DW_N2V_POS', '1') != '0'


def _graph_fingerprint(graph) -> int:
    """Hash of the adjacency in insertion order with edge weights: a rewired edge or a changed
    weight gives a new CSR (the reference reads the live graph on every step). O(E)."""
    return hash(tuple((n, tuple((x, d.get('weight')) for x, d in nbrs.items()))
                      for n, nbrs in graph.adj.items()))


def _csr_of(graph) -> CSRGraph:
    """CSR of a networkx graph, cached on the graph object (the walker borrows the graph) and
    rebuilt when the graph changed since (structure, neighbour order or weights)."""
    if isinstance(graph, CSRGraph):
        return graph
    key = _graph_fingerprint(graph)
    cached = graph.graph.get(_CSR_CACHE_ATTR) if hasattr(graph, 'graph') else None
    if cached is not None and cached[0] == key:
        return cached[1]
    csr = CSRGraph.from_networkx(graph)
    graph.graph[_CSR_CACHE_ATTR] = (key, csr)
    return csr


def _dyadic_scale(x: np.ndarray) -> int:
    """Smallest k >= 0 such that every finite double in ``x`` is a multiple of 2**-k."""
    x = np.abs(np.asarray(x, dtype=np.float64).reshape(-1))
    x = x[x > 0]
    if x.size == 0:
        return 0
    m, e = np.frexp(x)                                   # x = m * 2**e, m in [0.5, 1)
    mant = (m * 2.0 ** 53).astype(np.uint64)             # x = mant * 2**(e - 53), exactly
    low = mant & (~mant + np.uint64(1))                  # lowest set bit of the mantissa
    tz = np.log2(low.astype(np.float64)).astype(np.int64)
    return int(max(0, int(np.max(53 - e.astype(np.int64) - tz))))


def sum_is_exact(csr: CSRGraph, inv_p: float, inv_q: float, node2vec: bool) -> bool:
    """True when every left-to-right partial sum of every step's (modified) weights is exactly
    representable, so naive and compensated summation give the same double (random_walk_generator
    .py:50-53,110 ``sum(neighbor_weights)``): all terms are multiples of 2**-k and the largest
    row's total stays below 2**53 at that scale."""
    factors = [1.0, float(inv_p), float(inv_q)] if node2vec else [1.0]
    if not all(np.isfinite(factors)):
        return False
    row_ptr = np.asarray(csr.row_ptr, dtype=np.int64)
    deg = np.diff(row_ptr)
    if csr.weights is None:
        terms = np.asarray(factors, dtype=np.float64)
        k = _dyadic_scale(terms)
        bound = float(deg.max(initial=0)) * float(terms.max()) * 2.0 ** k
        return bound < 2.0 ** 53
    w = np.asarray(csr.weights, dtype=np.float64)
    if not np.all(np.isfinite(w)):
        return False
    terms = [w * f for f in factors]                     # fl(w * (1/p)): the reference's product
    k = max(_dyadic_scale(t) for t in terms)
    big = np.max(np.stack([np.abs(t) for t in terms]), axis=0) if w.size else w
    nz = deg > 0
    if not nz.any():
        return True
    row_tot = np.add.reduceat(big, row_ptr[:-1][nz]) if big.size else np.zeros(0)
    return float(row_tot.max(initial=0.0)) * 2.0 ** k < 2.0 ** 53


class RandomWalk(ABC):
    """RandomWalk method interface (random_walk_generator.py:11-53)."""
    METHOD = _native.DW_METHOD_DEEPWALK

    def __init__(self, graph, length: int, rng: str = 'python', seed: int = 0, device=None,
                 layout: str = 'indexed'):
        """
        Args:
            graph: ``networkx.Graph`` (or a prebuilt ``CSRGraph`` for large synthetic graphs)
            length: random walk length
            rng: 'python' (bit-exact replay of the global ``random`` stream) or 'philox'
            seed: Philox key (rng='philox')
            device: HIP device (default: current)
            layout: rng='philox' — 'indexed' (default: DeepWalk over the edge-inline CSR,
                dw_walk_fast_indexed, one dependent load per step; node2vec on an unweighted
                graph over the per-edge position index, dw_walk_fast_positions — one Philox
                uniform and a search of the step's positions, no rejection rounds — where the
                index is small enough — CSRGraph.philox_positions, decided from the graph's
                size alone — else as 'hash'), 'positions' (node2vec over the index whatever its
                size, e.g. C5's 132 GB; an error where it cannot be built), 'hash' (node2vec by
                rejection with the adjacency tests in the per-row hash, dw_walk_fast_indexed) or
                'csr' (dw_walk_fast: row_ptr / col, node2vec's tests by search of the sorted
                lists; the same walks as 'hash' bit for bit). The position walker samples the
                same law from a different use of the Philox stream. rng='python':
                'indexed' runs DeepWalk on unweighted graphs over the edge-inline CSR
                (dw_walk_replay_inline), 'csr' keeps dw_walk_replay; the same walks.
        """
        assert length >= 1, 'Minimum walk length is 1!'
        if rng not in ('python', 'philox'):
            raise ValueError(f'unknown rng "{rng}" (expected "python" or "philox")')
        if layout not in ('indexed', 'hash', 'csr', 'positions'):
            raise ValueError(f'unknown layout "{layout}" (expected "indexed", "hash", "csr" or '
                             f'"positions")')
        if layout == 'positions' and (rng != 'philox' or self.METHOD != _native.DW_METHOD_NODE2VEC):
            raise ValueError("layout='positions' is the Philox node2vec walker's")
        self.last_walker = None   # the kernel of the last walk_batch call
        self._layout = layout
        self._graph = graph
        self._length = length
        self._rng = rng
        self._seed = int(seed)
        self._device = device
        self._csr = _csr_of(graph)
        self._next_walk_id = 0
        self._check_sum_semantics()

    def _check_sum_semantics(self) -> None:
        """rng='python' on CPython >= 3.12: ``sum()`` of floats is compensated there (Neumaier),
        while the replay's serial fallback sums left to right as <= 3.11 does. The two agree
        whenever every partial sum of a step's weights is exact (``sum_is_exact``), which covers
        unweighted DeepWalk (int 1s), integer weights, and p, q whose reciprocals are short
        binary fractions (the BASELINE configs' 1, 2, 4, 0.25, 0.5); anything else raises."""
        if self._rng != 'python' or sys.version_info < (3, 12):
            return
        p, q = self._params()
        if not sum_is_exact(self._csr, 1.0 / p, 1.0 / q,
                            node2vec=self.METHOD == _native.DW_METHOD_NODE2VEC):
            raise NotImplementedError(
                "rng='python' (bit-exact replay) on CPython >= 3.12 needs step weights whose "
                "sums are exact (integer weights, reciprocals of p and q with short binary "
                "expansions): 3.12's compensated float sum() would round differently; use "
                "rng='philox' or CPython < 3.12")

    # ---- reference host helpers (random_walk_generator.py:41-53) -----------------------
    @property
    def csr(self) -> CSRGraph:
        return self._csr

    @property
    def length(self) -> int:
        return self._length

    def get_node_neighbors(self, node) -> List:
        if isinstance(self._graph, CSRGraph):
            return [self._csr.names[i] for i in self._csr.neighbors(self._csr.node_id(node))]
        return list(self._graph.neighbors(node))

    def get_node_unnormalized_edge_weights(self, node) -> List[float]:
        i = self._csr.node_id(node)
        a, b = self._csr.row_ptr[i], self._csr.row_ptr[i + 1]
        if self._csr.weights is None:
            return [1 for _ in range(a, b)]
        return [float(w) for w in self._csr.weights[a:b]]

    def get_node_normalized_edge_weights(self, node) -> List[float]:
        w = self.get_node_unnormalized_edge_weights(node)
        s = sum(w)
        return [x / s for x in w]

    # ---- walks ------------------------------------------------------------------------
    def _params(self):
        return 1.0, 1.0

    def walk(self, node) -> str:
        """Performs a random walk starting from ``node``; returns ``'n1 n2 n3'``."""
        ids = self.walk_batch(torch.tensor([self._csr.node_id(node)], dtype=torch.int32))
        return ' '.join(str(self._csr.names[i]) for i in ids[0].tolist())

    def walk_batch(self, start_ids: Union[torch.Tensor, Sequence[int]],
                   uniforms: Optional[np.ndarray] = None, walk_id0: Optional[int] = None,
                   out: Optional[torch.Tensor] = None, check: bool = True,
                   status: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Walks from every start id (vocabulary ids) — int32 [n, length] on the device.

        rng='python': the next n*(length-1) doubles of the global ``random`` stream are used,
        generated on the device (or ``uniforms`` when given, shape [n, length-1]; host or
        device). rng='philox': walk ``k`` of this
        call has global walk id ``walk_id0 + k`` (default: continues the previous call).
        ``check=False`` skips the synchronising status check (stream stays asynchronous);
        ``status``: the caller's int32 status word to OR conditions into (default: a new one).
        """
        dev = _native.require_device(self._device)
        starts = torch.as_tensor(start_ids, dtype=torch.int32)
        starts = starts.to(dev, non_blocking=True).contiguous()
        n = int(starts.numel())
        L = self._length
        n2v = self.METHOD == _native.DW_METHOD_NODE2VEC
        # replay: the CSR, adjacency by search of the sorted lists; philox: DeepWalk over the
        # edge-inline CSR, node2vec with the per-row adjacency hash (the same walks as
        # dw_walk_fast, bit for bit; layout='csr' selects that one)
        indexed = self._rng == 'philox' and self._layout in ('indexed', 'hash', 'positions')
        # Philox node2vec on an unweighted graph: over the position index where it fits
        pos_fast = self._positions_walker(dev)
        # replay, DeepWalk on an unweighted graph: the same walks over the edge-inline CSR
        # (dw_walk_replay_inline; layout='csr' keeps dw_walk_replay)
        replay_inline = (self._rng == 'python' and not n2v and self._layout == 'indexed'
                         and self._csr.weights is None)
        # replay, node2vec on an unweighted graph: the adjacency-hash replay (dw_walk_replay_
        # indexed: the shorter list of each step probed; the same walks as dw_walk_replay)
        replay_n2v_idx = (self._rng == 'python' and n2v and self._layout == 'indexed'
                          and self._csr.weights is None)
        d = self._csr.device_tensors(dev, need_sorted=n2v and not indexed,
                                     need_alias=self._rng == 'philox',
                                     need_edges=(indexed and not n2v) or replay_inline,
                                     need_adj=indexed and n2v and not pos_fast,
                                     need_adj_pos=replay_n2v_idx,
                                     need_hub_bits=replay_n2v_idx,
                                     need_edge_cn=replay_n2v_idx and _edge_cn_enabled(),
                                     need_n2v_index=replay_n2v_idx and _n2v_index_enabled())
        if self._rng == 'python' and n2v:
            self._csr.require_simple(dev)   # no repeated neighbour (nx.Graph's invariant)
        if out is None:
            out = torch.empty((n, L), dtype=torch.int32, device=dev)
        if status is None:
            status = torch.zeros(1, dtype=torch.int32, device=dev)
        p, q = self._params()
        with torch.cuda.device(dev):
            s = _native.stream(dev)
            commit = None
            if self._rng == 'python':
                if uniforms is None:   # the global stream, made in HBM; committed after launch
                    uniforms, commit = draw_uniforms_device(n * (L - 1), dev, defer=True)
                if isinstance(uniforms, torch.Tensor):   # e.g. already resident on the device
                    u = uniforms.reshape(-1).to(device=dev, dtype=torch.float64).contiguous()
                else:
                    u = torch.from_numpy(np.ascontiguousarray(uniforms,
                                                              dtype=np.float64).reshape(-1))
                if u.numel() != n * (L - 1):
                    raise ValueError('uniforms must have n_walks * (length - 1) values')
                u = u.to(dev)
                if replay_inline:
                    self.last_walker = 'dw_walk_replay_inline'
                    _native.call('dw_walk_replay_inline', _native.ptr(d['row_ptr']),
                                 _native.ptr(d['edges']), self._csr.vocab_size,
                                 _native.ptr(starts), n, L,
                                 _native.ptr(u) if u.numel() else None, _native.ptr(out),
                                 _native.ptr(status), s)
                elif replay_n2v_idx:
                    self._replay_n2v(d, starts, n, u, out, status, None, s)
                else:
                    self.last_walker = 'dw_walk_replay'
                    _native.call('dw_walk_replay', _native.ptr(d['row_ptr']),
                                 _native.ptr(d['col']), _native.ptr(d.get('col_sorted')),
                                 _native.ptr(d['weights']), self._csr.vocab_size,
                                 _native.ptr(starts), n, L, self.METHOD, float(p), float(q),
                                 _native.ptr(u) if u.numel() else None, _native.ptr(out),
                                 _native.ptr(status), s)
                if commit is not None:
                    commit()
            else:
                wid0 = self._next_walk_id if walk_id0 is None else int(walk_id0)
                if pos_fast:
                    self.last_walker = 'dw_walk_fast_positions'
                    _native.call('dw_walk_fast_positions', _native.ptr(d['row_ptr']),
                                 _native.ptr(d['n2v_rec']), _native.ptr(d['n2v_pos']),
                                 self._csr.vocab_size, _native.ptr(starts), n, L, float(p),
                                 float(q), self._seed & 0xFFFFFFFFFFFFFFFF, wid0,
                                 _native.ptr(out), _native.ptr(status), None, s)
                elif indexed:
                    self.last_walker = 'dw_walk_fast_indexed'
                    _native.call('dw_walk_fast_indexed', _native.ptr(d['row_ptr']),
                                 _native.ptr(d['col']), _native.ptr(d.get('edges')),
                                 _native.ptr(d.get('adj_off')), _native.ptr(d.get('adj_hash')),
                                 _native.ptr(d.get('prob_thr')),
                                 _native.ptr(d.get('alias')), self._csr.vocab_size,
                                 _native.ptr(starts), n, L, self.METHOD, float(p), float(q),
                                 self._seed & 0xFFFFFFFFFFFFFFFF, wid0, _native.ptr(out),
                                 _native.ptr(status), s)
                else:
                    self.last_walker = 'dw_walk_fast'
                    _native.call('dw_walk_fast', _native.ptr(d['row_ptr']), _native.ptr(d['col']),
                                 _native.ptr(d.get('col_sorted')), _native.ptr(d.get('prob_thr')),
                                 _native.ptr(d.get('alias')), self._csr.vocab_size,
                                 _native.ptr(starts), n, L, self.METHOD, float(p), float(q),
                                 self._seed & 0xFFFFFFFFFFFFFFFF, wid0, _native.ptr(out),
                                 _native.ptr(status), s)
                self._next_walk_id = wid0 + n
        if check:
            _native.check_status(status, f'{type(self).__name__}.walk')
        return out

    def _positions_walker(self, dev) -> bool:
        """rng='philox', node2vec: True when dw_walk_fast_positions walks — layout='positions'
        (the index built whatever its size, or an error), or layout='indexed' on a graph whose
        index is small enough (CSRGraph.philox_positions: decided once per graph from its size,
        never from the device's free memory, so the same seed gives the same walks on any
        device); else the rejection walker over the adjacency hash."""
        if not (self._rng == 'philox' and self.METHOD == _native.DW_METHOD_NODE2VEC):
            return False
        if self._layout == 'positions':
            self._csr.require_n2v_index(dev)
            return True
        return self._layout == 'indexed' and self._csr.philox_positions(dev)

    def count_replay_traffic(self, start_ids: torch.Tensor, uniforms: torch.Tensor,
                             out: Optional[torch.Tensor] = None) -> dict:
        """node2vec, rng='python', unweighted: the same walks as ``walk_batch(start_ids,
        uniforms)`` with the replay walker's realised traffic counted (dw_walk_replay_indexed
        with counters; a diagnostic launch): {'bytes', 'probes', 'entries', 'steps'} (over the
        position index: 'probes' counts the picks made by the serial arithmetic, 'entries' the
        2-B position units read, 'lines' the searches' dependent 128-B line moves)."""
        if self.METHOD != _native.DW_METHOD_NODE2VEC or self._rng != 'python' \
                or self._csr.weights is not None:
            raise ValueError('count_replay_traffic: node2vec with rng="python", unweighted')
        dev = _native.require_device(self._device)
        starts = torch.as_tensor(start_ids, dtype=torch.int32).to(dev).contiguous()
        n, L = int(starts.numel()), self._length
        u = torch.as_tensor(uniforms).reshape(-1).to(device=dev, dtype=torch.float64).contiguous()
        if u.numel() != n * (L - 1):
            raise ValueError('uniforms must have n_walks * (length - 1) values')
        d = self._csr.device_tensors(dev, need_sorted=True, need_adj_pos=True,
                                     need_hub_bits=True, need_edge_cn=_edge_cn_enabled(),
                                     need_n2v_index=_n2v_index_enabled())
        self._csr.require_simple(dev)
        if out is None:
            out = torch.empty((n, L), dtype=torch.int32, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        counters = torch.zeros(5, dtype=torch.int64, device=dev)
        with torch.cuda.device(dev):
            self._replay_n2v(d, starts, n, u, out, status, counters, _native.stream(dev))
        _native.check_status(status, f'{type(self).__name__}.count_replay_traffic')
        c = counters.cpu().tolist()
        return {'bytes': c[0], 'probes': c[1], 'entries': c[2], 'steps': c[3], 'lines': c[4]}

    def _replay_n2v(self, d, starts, n, u, out, status, counters, s) -> None:
        """The exact node2vec walks on an unweighted graph: over the position index when it is
        built (dw_walk_replay_positions), else the wave walker (dw_walk_replay_indexed)."""
        L = self._length
        p, q = self._params()
        common = [_native.ptr(d['row_ptr']), _native.ptr(d['col']), _native.ptr(d['col_sorted']),
                  _native.ptr(d['adj_off']), _native.ptr(d['adj_hash']),
                  _native.ptr(d['adj_hpos']), _native.ptr(d['hub_idx']),
                  _native.ptr(d['hub_bits']), d['hub_words'],
                  _native.ptr(d.get('edge_cn') if _edge_cn_enabled() else None)]
        uptr = _native.ptr(u) if u.numel() else None
        if _n2v_index_enabled() and d.get('n2v_rec') is not None:
            self.last_walker = 'dw_walk_replay_positions'
            _native.call('dw_walk_replay_positions', _native.ptr(d['row_ptr']),
                         _native.ptr(d['n2v_rec']), _native.ptr(d['n2v_pos']),
                         self._csr.vocab_size, _native.ptr(starts), n, L, float(p), float(q),
                         uptr, _native.ptr(out), _native.ptr(status), _native.ptr(counters), s)
            return
        self.last_walker = 'dw_walk_replay_indexed'
        _native.call('dw_walk_replay_indexed', *common, self._csr.vocab_size,
                     _native.ptr(starts), n, L, float(p), float(q), uptr, _native.ptr(out),
                     _native.ptr(status), _native.ptr(counters), s)

    def count_traffic(self, start_ids: torch.Tensor, walk_id0: int,
                      out: Optional[torch.Tensor] = None) -> dict:
        """node2vec, rng='philox', layout='indexed': the same walks as ``walk_batch`` with the
        walkers' realised memory traffic counted (dw_walk_fast_counted; a diagnostic launch):
        {'bytes', 'steps', 'blocks', 'tests'} summed over the walks."""
        if self.METHOD != _native.DW_METHOD_NODE2VEC or self._rng != 'philox' \
                or self._layout not in ('indexed', 'hash', 'positions'):
            raise ValueError('count_traffic: node2vec with rng="philox", layout="indexed" or '
                             '"hash"')
        dev = _native.require_device(self._device)
        starts = torch.as_tensor(start_ids, dtype=torch.int32).to(dev).contiguous()
        n, L = int(starts.numel()), self._length
        if self._positions_walker(dev):   # {'bytes', 'steps', 0, position 2-B units read}
            d = self._csr.device_tensors(dev)
            if out is None:
                out = torch.empty((n, L), dtype=torch.int32, device=dev)
            status = torch.zeros(1, dtype=torch.int32, device=dev)
            counters = torch.zeros(4, dtype=torch.int64, device=dev)
            p, q = self._params()
            with torch.cuda.device(dev):
                _native.call('dw_walk_fast_positions', _native.ptr(d['row_ptr']),
                             _native.ptr(d['n2v_rec']), _native.ptr(d['n2v_pos']),
                             self._csr.vocab_size, _native.ptr(starts), n, L, float(p), float(q),
                             self._seed & 0xFFFFFFFFFFFFFFFF, int(walk_id0), _native.ptr(out),
                             _native.ptr(status), _native.ptr(counters), _native.stream(dev))
            _native.check_status(status, f'{type(self).__name__}.count_traffic')
            c = counters.cpu().tolist()
            return {'bytes': c[0], 'steps': c[1], 'blocks': 0, 'tests': 0,
                    'position_loads': c[3], 'position_lines': c[2],
                    'walker': 'dw_walk_fast_positions'}
        d = self._csr.device_tensors(dev, need_alias=True, need_adj=True)
        if out is None:
            out = torch.empty((n, L), dtype=torch.int32, device=dev)
        status = torch.zeros(1, dtype=torch.int32, device=dev)
        counters = torch.zeros(4, dtype=torch.int64, device=dev)
        p, q = self._params()
        with torch.cuda.device(dev):
            _native.call('dw_walk_fast_counted', _native.ptr(d['row_ptr']), _native.ptr(d['col']),
                         _native.ptr(d['adj_off']), _native.ptr(d['adj_hash']),
                         _native.ptr(d.get('prob_thr')), _native.ptr(d.get('alias')),
                         self._csr.vocab_size, _native.ptr(starts), n, L, float(p), float(q),
                         self._seed & 0xFFFFFFFFFFFFFFFF, int(walk_id0), _native.ptr(out),
                         _native.ptr(status), _native.ptr(counters), _native.stream(dev))
        _native.check_status(status, f'{type(self).__name__}.count_traffic')
        c = counters.cpu().tolist()
        return {'bytes': c[0], 'steps': c[1], 'blocks': c[2], 'tests': c[3]}


class DeepWalk(RandomWalk):
    """First-order walk (random_walk_generator.py:56-72). https://arxiv.org/pdf/1403.6652.pdf"""
    METHOD = _native.DW_METHOD_DEEPWALK


class Node2Vec(RandomWalk):
    """Second-order (p, q) walk (random_walk_generator.py:75-119).

    Reproduces the reference's rule exactly, including its inversion of the paper's q:
    a candidate equal to the previous node gets ``w * (1/p)``; a candidate ADJACENT to the
    previous node gets ``w * (1/q)``; distance-2 candidates keep ``w``
    (random_walk_generator.py:101-108). https://arxiv.org/pdf/1607.00653.pdf
    """
    METHOD = _native.DW_METHOD_NODE2VEC

    def __init__(self, graph, length: int, p: float = 1.0, q: float = 1.0, **kwargs):
        self._p = p      # set first: the base constructor's sum check reads them
        self._q = q
        super().__init__(graph=graph, length=length, **kwargs)

    def _params(self):
        return self._p, self._q


def random_walk_factory(name: str, graph, length: int,
                        additional_params: Optional[dict] = None, **walker_kwargs) -> RandomWalk:
    """Creates a random walk generator by name (random_walk_generator.py:122-151).

    ``walker_kwargs`` (rng, seed, device) select the sampling mode; method parameters (p, q)
    come through ``additional_params`` exactly as in the reference.
    """
    name = name.lower()
    if additional_params is None:
        additional_params = {}

    SUPPORTED_METHODS = {
        'deepwalk': DeepWalk,
        'dfs': DeepWalk,
        'node2vec': Node2Vec,
    }
    assert name in SUPPORTED_METHODS, \
        f'Unknown method "{name}". Supported: {list(SUPPORTED_METHODS.keys())}'
    return SUPPORTED_METHODS[name](graph=graph, length=length, **additional_params,
                                   **walker_kwargs)

