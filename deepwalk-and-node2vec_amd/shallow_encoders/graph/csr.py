"""CSR adjacency in vocabulary-id space — the device layout of the reference's networkx graph.

The reference walks a ``networkx.Graph`` from Python (random_walk_generator.py:41-48) and maps
node names to ids through a torchtext vocabulary built from one extra epoch of walks
(torch_dataset.py:91-110: ``<unk>`` first, then tokens sorted lexicographically since every
node occurs once). Here the vocabulary is built directly from the node names with the same
rule, and the adjacency becomes

    row_ptr int64[V+1]   row 0 = ``<unk>`` (no neighbours), row i = node with vocab id i
    col     int32[nnz]   neighbour ids in ``graph.neighbors(node)`` order (insertion order)
    weights float64[nnz] the ``'weight'`` attribute when ``nx.is_weighted(graph)``, else None
    col_sorted int32[nnz] each row ascending (device-built by dw_csr_sort_copy), for the
                          node2vec adjacency test ``prev_node in candidate_neighbors``.
"""
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from shallow_encoders import _native

UNK = '<unk>'
_TOKEN_RE = re.compile(r"[A-Za-z]+[\w^']*|[\w^']*[A-Za-z]+[\w^']*|<unk>")


def node_token(name) -> str:
    """The vocabulary token of a node name (reference tokenizer, torch_dataset.py:23-39).

    A node name must tokenize to exactly one token (the reference joins walk names with
    spaces and re-tokenizes them); names such as ``'a b'`` or ``'1'`` cannot round-trip.
    """
    s = str(name)
    toks = _TOKEN_RE.findall(s.lower())
    if len(toks) != 1 or toks[0] != s.lower():
        raise ValueError(f'node name {s!r} does not tokenize to a single vocabulary token '
                         f'(got {toks}); node names must start with a letter')
    return toks[0]


class NodeNames(Sequence):
    """``['<unk>', 'n0000000', 'n0000001', ...]`` computed on demand (synthetic graphs: node i
    is named n%0{width}d and has vocabulary id i + 1), so a 16.8M-node graph does not hold
    16.8M Python strings."""

    def __init__(self, n_nodes: int, width: int):
        self.n, self.width = int(n_nodes), int(width)

    def __len__(self) -> int:
        return self.n + 1

    def _name(self, i: int) -> str:
        return UNK if i == 0 else f'n{i - 1:0{self.width}d}'

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._name(j) for j in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._name(i)

    def index(self, token, *args) -> int:
        m = re.fullmatch(r'n(\d+)', str(token))
        if token == UNK:
            return 0
        if m is None or len(m.group(1)) != self.width or int(m.group(1)) >= self.n:
            raise ValueError(f'{token!r} is not a node name')
        return int(m.group(1)) + 1


@dataclass
class CSRGraph:
    """Host (numpy) CSR plus lazily built device copies."""
    row_ptr: np.ndarray                 # int64 [V+1]
    col: np.ndarray                     # int32 [nnz]
    weights: Optional[np.ndarray]       # float64 [nnz] or None
    itos: List[str]                     # vocabulary (id -> token), itos[0] == '<unk>'
    names: List[object]                 # id -> original node object (None for <unk>)
    _dev: Dict[str, torch.Tensor] = field(default_factory=dict, repr=False)
    _dev_device: Optional[torch.device] = field(default=None, repr=False)

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_networkx(graph) -> 'CSRGraph':
        import networkx as nx
        nodes = list(graph)
        tokens = [node_token(n) for n in nodes]
        if len(set(tokens)) != len(tokens):
            raise ValueError('two node names map to the same vocabulary token')
        itos = [UNK] + sorted(tokens)
        stoi = {t: i for i, t in enumerate(itos)}
        names: List[object] = [None] * len(itos)
        for n, t in zip(nodes, tokens):
            names[stoi[t]] = n
        weighted = nx.is_weighted(graph) if graph.number_of_edges() > 0 else False
        V = len(itos)
        deg = np.zeros(V, dtype=np.int64)
        rows = [None] * V
        wrows = [None] * V
        adj = graph.adj
        for n, t in zip(nodes, tokens):
            i = stoi[t]
            nbrs = adj[n]
            rows[i] = [stoi[node_token(x)] for x in nbrs]
            if weighted:
                wrows[i] = [float(nbrs[x]['weight']) for x in nbrs]
            deg[i] = len(rows[i])
        row_ptr = np.zeros(V + 1, dtype=np.int64)
        np.cumsum(deg, out=row_ptr[1:])
        col = np.empty(int(row_ptr[-1]), dtype=np.int32)
        w = np.empty(int(row_ptr[-1]), dtype=np.float64) if weighted else None
        for i in range(1, V):
            a, b = row_ptr[i], row_ptr[i + 1]
            col[a:b] = rows[i]
            if weighted:
                w[a:b] = wrows[i]
        return CSRGraph(row_ptr, col, w, itos, names)

    @staticmethod
    def from_arrays(row_ptr, col, weights=None, itos: Optional[Sequence[str]] = None,
                    names: Optional[Sequence[object]] = None) -> 'CSRGraph':
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.int64)
        col = np.ascontiguousarray(col, dtype=np.int32)
        weights = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
        V = len(row_ptr) - 1
        if itos is None:
            width = max(7, len(str(V - 1)))
            itos = [UNK] + [f'n{i:0{width}d}' for i in range(V - 1)]
        if not isinstance(itos, NodeNames):
            itos = list(itos)
        if names is None:
            names = itos if isinstance(itos, NodeNames) else [None] + itos[1:]
        if len(itos) != V:
            raise ValueError('itos length must equal the number of CSR rows')
        return CSRGraph(row_ptr, col, weights, itos,
                        names if isinstance(names, NodeNames) else list(names))

    @staticmethod
    def from_device(row_ptr: torch.Tensor, col: torch.Tensor, itos: Sequence[str]) -> 'CSRGraph':
        """A CSR built in HBM (dw_csr_from_edges): row_ptr is copied to the host (V+1 int64),
        col stays on the device only (``col`` is None until ``host_col()``)."""
        g = CSRGraph(row_ptr.cpu().numpy(), None, None, itos, itos)
        g._dev_device = col.device
        g._dev = {'row_ptr': row_ptr, 'col': col, 'weights': None,
                  'status': torch.zeros(1, dtype=torch.int32, device=col.device)}
        return g

    def host_col(self) -> np.ndarray:
        """The column array on the host (downloaded once for device-built graphs)."""
        if self.col is None:
            self.col = self._dev['col'].cpu().numpy()
        return self.col

    # ------------------------------------------------------------------ host helpers
    @property
    def vocab_size(self) -> int:
        return len(self.row_ptr) - 1

    @property
    def nnz(self) -> int:
        return int(self.row_ptr[-1])

    @property
    def weighted(self) -> bool:
        return self.weights is not None

    def degree(self) -> np.ndarray:
        return np.diff(self.row_ptr)

    def neighbors(self, i: int) -> np.ndarray:
        return self.host_col()[self.row_ptr[i]:self.row_ptr[i + 1]]

    def stoi(self) -> Dict[str, int]:
        return {t: i for i, t in enumerate(self.itos)}

    def node_id(self, node) -> int:
        tok = node_token(node)
        if isinstance(self.itos, NodeNames):
            return self.itos.index(tok)
        sto = self.__dict__.setdefault('_stoi_cache', None)
        if sto is None:
            sto = self.stoi()
            self.__dict__['_stoi_cache'] = sto
        return sto[tok]

    # ------------------------------------------------------------------ device side
    def device_tensors(self, device=None, need_sorted: bool = False,
                       need_alias: bool = False, need_edges: bool = False,
                       need_adj: bool = False, need_adj_pos: bool = False,
                       need_hub_bits: bool = False,
                       need_edge_cn: bool = False,
                       need_n2v_index: bool = False,
                       n2v_budget: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """Copy the CSR to HBM once (and derive col_sorted / alias tables / the edge-inline CSR /
        the per-row adjacency hash / its slots' neighbour positions on the device)."""
        dev = _native.require_device(device)
        if self._dev_device != dev:
            if self.col is None and 'col' in self._dev:   # device-built: keep a host copy
                self.col = self._dev['col'].cpu().numpy()
            self._dev = {}
            self._dev_device = dev
        d = self._dev
        if 'row_ptr' not in d:
            d['row_ptr'] = torch.from_numpy(self.row_ptr).to(dev)
            d['col'] = torch.from_numpy(self.host_col()).to(dev)
            d['weights'] = None if self.weights is None else torch.from_numpy(self.weights).to(dev)
            d['status'] = torch.zeros(1, dtype=torch.int32, device=dev)
            st = d['status']
            with torch.cuda.device(dev):
                _native.call('dw_csr_validate', _native.ptr(d['row_ptr']),
                             _native.ptr(d['col']) if self.nnz else None, self.vocab_size,
                             self.nnz, _native.ptr(st), _native.stream(dev))
            _native.check_status(st, 'CSR validation')
        if need_sorted and 'col_sorted' not in d:
            d['col_sorted'] = self._sorted_copy(dev)
        if need_alias and self.weights is not None and 'prob_thr' not in d:
            self._build_alias(dev)
        if need_edges and 'edges' not in d:
            self._build_edges(dev)
        if (need_adj or need_adj_pos or need_edge_cn) and 'adj_off' not in d:
            self._build_adj_hash(dev)
        if need_adj_pos and 'adj_hpos' not in d:
            n_slots = d['adj_hash'].numel()
            hp = torch.empty(n_slots, dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                _native.call('dw_adj_hash_positions', _native.ptr(d['row_ptr']),
                             _native.ptr(d['col']) if self.nnz else None, self.vocab_size,
                             _native.ptr(d['adj_off']), _native.ptr(d['adj_hash']),
                             int(d['adj_off'][self.vocab_size]), _native.ptr(hp),
                             _native.ptr(d['status']), _native.stream(dev))
            _native.check_status(d['status'], 'adjacency positions build')
            d['adj_hpos'] = hp
        if need_hub_bits and 'hub_idx' not in d:
            self._build_hub_bits(dev)
        if need_edge_cn and 'edge_cn' not in d:
            if 'adj_hpos' not in d or 'hub_idx' not in d:
                self.device_tensors(dev, need_adj_pos=True, need_hub_bits=True)
            cn = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                _native.call('dw_edge_common_counts', _native.ptr(d['row_ptr']),
                             _native.ptr(d['col']) if self.nnz else None,
                             _native.ptr(d['adj_off']), _native.ptr(d['adj_hash']),
                             _native.ptr(d['adj_hpos']), _native.ptr(d['hub_idx']),
                             _native.ptr(d['hub_bits']), d['hub_words'], self.vocab_size,
                             self.nnz, _native.ptr(cn), _native.stream(dev))
            d['edge_cn'] = cn
        if need_n2v_index:
            info = d.get('n2v_index_info') or {}
            # a skipped index is tried again only when a larger cap is asked for (the exact
            # walker's default after a smaller explicit one) — not because free memory grew (an
            # out-of-memory skip empties the cache, which would retry the whole build at every
            # call) and never inside a graph capture
            cap = self.N2V_INDEX_BYTES if n2v_budget is None else int(n2v_budget)
            if 'n2v_rec' not in d or (d['n2v_rec'] is None and cap > info.get('cap', 0)
                                      and not info.get('unsupported')
                                      and not torch.cuda.is_current_stream_capturing()):
                self._build_n2v_index(dev, n2v_budget)
        return d

    def philox_positions(self, device=None) -> bool:
        """Whether rng='philox' node2vec (layout='indexed') walks over the position index
        (dw_walk_fast_positions) or by rejection (dw_walk_fast_indexed) on this graph: the two
        use the Philox stream differently, so they give different walks, and the choice must not
        depend on the device's free memory. It is decided once per graph and device from the
        graph alone — the index's size (entries + records, a function of the graph) against
        N2V_PHILOX_INDEX_BYTES — and cached; the index is then built without the free-memory
        cap (torch.OutOfMemoryError if it cannot be; layout='hash' selects the rejection walker
        explicitly). Weighted graphs and rows with a repeated neighbour keep the rejection
        walker."""
        dev = _native.require_device(device)
        d = self.device_tensors(dev)
        if 'philox_positions' in d:
            return d['philox_positions']
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError('the Philox node2vec walker is chosen (and its index built) '
                               'before a graph capture: walk once first')
        use = False
        if self.weights is None and self.is_simple(dev) and 16 * (self.nnz + 1) <= \
                self.N2V_PHILOX_INDEX_BYTES:
            info = d.get('n2v_index_info') or {}
            if 'bytes' not in info:   # the size is known once the offsets have been scanned
                self._build_n2v_index(dev, self.N2V_PHILOX_INDEX_BYTES, fixed=True)
                info = d['n2v_index_info']
            use = not info.get('unsupported') and info['bytes'] <= self.N2V_PHILOX_INDEX_BYTES
            if use and d.get('n2v_rec') is None:
                self._build_n2v_index(dev, info['bytes'], fixed=True)
        d['philox_positions'] = use
        return use

    def require_n2v_index(self, device=None) -> Dict[str, torch.Tensor]:
        """The position index built whatever its size (layout='positions'): OutOfMemoryError
        when the device cannot hold it, ValueError on a weighted graph or a repeated
        neighbour."""
        dev = _native.require_device(device)
        if self.weights is not None:
            raise ValueError('the node2vec position index needs an unweighted graph')
        self.require_simple(dev)
        d = self.device_tensors(dev)
        if d.get('n2v_rec') is None:
            self._build_n2v_index(dev, 1 << 62, fixed=True)
            if d.get('n2v_rec') is None:
                raise ValueError(f'the node2vec position index cannot be built for this graph: '
                                 f'{d.get("n2v_index_info")}')
        return d

    # the position index is built when its entries, records and build scratch fit this many
    # bytes and the device's free memory less a reserve (DW_N2V_INDEX_BYTES overrides both);
    # above it the walker keeps the counted classification
    N2V_INDEX_BYTES = 192 << 30
    N2V_INDEX_RESERVE = 16 << 30
    # entries sorted per build launch (the scratch: 8 B each plus the sort's storage)
    N2V_CHUNK_ENTRIES = 1 << 28
    # the Philox walker's budget: it has the rejection walker to fall back on, so it builds the
    # index only where it is small next to the device (C3's 4 GB, not C5's 150: that memory
    # belongs to the training tables)
    N2V_PHILOX_INDEX_BYTES = 32 << 30

    def _n2v_budget(self, dev, budget: Optional[int]) -> int:
        """The byte budget of the position index: ``budget`` (None: N2V_INDEX_BYTES), capped at
        the device's free memory less N2V_INDEX_RESERVE; DW_N2V_INDEX_BYTES overrides both."""
        import os
        env = os.environ.get('DW_N2V_INDEX_BYTES')
        if env is not None:
            return int(env)
        cap = self.N2V_INDEX_BYTES if budget is None else int(budget)
        return min(cap, torch.cuda.mem_get_info(dev)[0] - self.N2V_INDEX_RESERVE)

    def _build_n2v_index(self, dev, budget: Optional[int] = None, fixed: bool = False) -> None:
        """n2v_rec int32[nnz, 8] / n2v_pos uint8[bytes] (dw_n2v_edge_offsets +
        dw_n2v_edge_index_build + dw_n2v_edge_records): per directed edge t -> v, t's position in
        N(v) and the sorted positions of N(t) ∩ N(v) — uint16 where deg(v) <= 65536, else int32 —
        the exact node2vec pick's binary search (dw_walk_replay_positions,
        dw_walk_fast_positions). Built in chunks of about N2V_CHUNK_ENTRIES entries, so the
        scratch stays bounded while the index grows to the graph's size (C5: 132 GB). Both None
        when the index would exceed the byte budget; n2v_index_info = {'entries', 'bytes',
        'chunks', 'budget', 'build_ms'} or {'entries', 'bytes', 'skipped', 'budget'}; ``budget``:
        its byte budget (_n2v_budget). ``fixed`` (philox_positions): the index is built when its
        own bytes fit ``budget``, whatever the device's free memory, and an allocation failure
        raises instead of skipping."""
        import ctypes
        import time
        d = self.device_tensors(dev, need_edge_cn=True)
        E = self.nnz
        colp = _native.ptr(d['col']) if E else None
        budget_b = int(budget) if fixed else self._n2v_budget(dev, budget)
        cap = self.N2V_INDEX_BYTES if budget is None else int(budget)
        with torch.cuda.device(dev):
            s = _native.stream(dev)
            t0 = time.perf_counter()
            nb = ctypes.c_size_t(0)
            try:   # (the offsets: 16 B per edge, before the index's size is known)
                if 16 * (E + 1) > budget_b:
                    raise torch.OutOfMemoryError('the offsets alone exceed the budget')
                off = torch.empty(E + 1, dtype=torch.int64, device=dev)
                boff = torch.empty(E + 1, dtype=torch.int64, device=dev)
                oargs = [_native.ptr(d['row_ptr']), colp, _native.ptr(d['edge_cn']), E,
                         _native.ptr(off), _native.ptr(boff)]
                _native.call('dw_n2v_edge_offsets', *oargs, None, ctypes.byref(nb), s)
                tmp = torch.empty(max(int(nb.value), 1), dtype=torch.uint8, device=dev)
            except torch.OutOfMemoryError:   # the wave walker needs none of it
                if fixed:
                    raise
                d['n2v_rec'], d['n2v_pos'] = None, None
                d['n2v_index_info'] = {'skipped': True, 'out_of_memory': True,
                                       'budget': budget_b, 'cap': cap}
                torch.cuda.empty_cache()
                return
            _native.call('dw_n2v_edge_offsets', *oargs, _native.ptr(tmp), ctypes.byref(nb), s)
            del tmp
            n_pos, n_bytes = (int(x) for x in torch.stack([off[E], boff[E]]).tolist())
            # chunk c = the edges [e_c, e_{c+1}), e_c = the first edge whose entries start at or
            # after c * K: at most K + max C(e) entries each
            K = self.N2V_CHUNK_ENTRIES
            cuts = torch.arange(0, max(n_pos, 1), K, dtype=torch.int64, device=dev)
            starts = torch.searchsorted(off, cuts).clamp_(max=E)
            bounds = torch.unique(torch.cat([starts, torch.tensor([0, E], device=dev)]))
            b_host = bounds.tolist()
            o_host = off[bounds].tolist()
            chunks = [(b_host[k], b_host[k + 1], o_host[k], o_host[k + 1] - o_host[k])
                      for k in range(len(b_host) - 1)]
            max_pos = max([c[3] for c in chunks] + [0])
            fits = E < (1 << 31) and max_pos < (1 << 31)
            tmp_need = 1
            args = [_native.ptr(d['row_ptr']), colp, _native.ptr(d['adj_off']),
                    _native.ptr(d['adj_hash']), _native.ptr(d['adj_hpos']),
                    _native.ptr(d['hub_idx']), _native.ptr(d['hub_bits']), d['hub_words'],
                    _native.ptr(d['edge_cn']), _native.ptr(off), _native.ptr(boff),
                    self.vocab_size, E]
            if fits:
                for e0, e1, base, cnt in chunks:
                    _native.call('dw_n2v_edge_index_build', *args, e0, e1, base, cnt, None, None,
                                 None, None, ctypes.byref(nb), None, s)
                    tmp_need = max(tmp_need, int(nb.value))
            index_bytes = n_bytes + 32 * E
            need = index_bytes + 4 * E + 4 * max_pos + tmp_need
            skipped = {'entries': n_pos, 'bytes': index_bytes, 'build_bytes': need,
                       'skipped': True, 'budget': budget_b, 'cap': cap,
                       'unsupported': not fits}
            if not fits or (index_bytes if fixed else need) > budget_b:
                d['n2v_rec'], d['n2v_pos'] = None, None
                d['n2v_index_info'] = skipped
                return
            try:
                pos = torch.empty(max(n_bytes, 4), dtype=torch.uint8, device=dev)
                rec = torch.empty((max(E, 1), 8), dtype=torch.int32, device=dev)
                pos_t = torch.empty(max(E, 1), dtype=torch.int32, device=dev)
                scratch = torch.empty(max(max_pos, 1), dtype=torch.int32, device=dev)
                tmp = torch.empty(tmp_need, dtype=torch.uint8, device=dev)
            except torch.OutOfMemoryError:   # the wave walker needs none of it
                if fixed:
                    raise
                d['n2v_rec'], d['n2v_pos'] = None, None
                d['n2v_index_info'] = dict(skipped, out_of_memory=True)
                torch.cuda.empty_cache()
                return
            for e0, e1, base, cnt in chunks:
                nb.value = tmp_need
                _native.call('dw_n2v_edge_index_build', *args, e0, e1, base, cnt,
                             _native.ptr(pos), _native.ptr(scratch), _native.ptr(pos_t),
                             _native.ptr(tmp), ctypes.byref(nb), _native.ptr(d['status']), s)
            del tmp, scratch
            _native.call('dw_n2v_edge_records', _native.ptr(d['row_ptr']), colp,
                         _native.ptr(d['edge_cn']), _native.ptr(boff), _native.ptr(pos_t), E,
                         _native.ptr(rec), s)
            del pos_t, off, boff
            _native.check_status(d['status'], 'node2vec position index build')
            d['n2v_rec'], d['n2v_pos'] = rec, pos
            d['n2v_index_info'] = {'entries': n_pos, 'bytes': index_bytes,
                                   'build_bytes': need, 'cap': cap,
                                   'chunks': len(chunks), 'budget': budget_b,
                                   'build_ms': (time.perf_counter() - t0) * 1e3}

    # rows longer than the replay walker's LDS stage (1,024) get a V-bit neighbour map, the
    # longest first, within this many bytes (DW_HUB_BITS_BYTES overrides)
    HUB_MIN_DEGREE = 1024
    HUB_BITS_BYTES = 2 << 30

    def _build_hub_bits(self, dev) -> None:
        """hub_idx int32[V] (-1 or the row's bitmap) / hub_bits int32[n_hubs, ceil(V/32)]
        (dw_hub_bitmaps): the bit-exact node2vec replay's membership tests against a hub."""
        import os
        d = self._dev
        V = self.vocab_size
        words = (V + 31) // 32
        budget = int(os.environ.get('DW_HUB_BITS_BYTES', self.HUB_BITS_BYTES))
        min_deg = int(os.environ.get('DW_HUB_MIN_DEGREE', self.HUB_MIN_DEGREE))
        deg = d['row_ptr'][1:] - d['row_ptr'][:-1]
        order = torch.argsort(deg, descending=True)
        n_big = int((deg > min_deg).sum())
        n_hubs = max(0, min(n_big, budget // max(1, words * 4)))
        hubs = order[:n_hubs].to(torch.int32).contiguous()
        idx = torch.full((V,), -1, dtype=torch.int32, device=dev)
        bits = torch.empty((max(n_hubs, 1), words), dtype=torch.int32, device=dev)
        if n_hubs:
            idx[hubs.long()] = torch.arange(n_hubs, dtype=torch.int32, device=dev)
            with torch.cuda.device(dev):
                _native.call('dw_hub_bitmaps', _native.ptr(d['row_ptr']), _native.ptr(d['col']),
                             V, _native.ptr(hubs), n_hubs, words, _native.ptr(bits),
                             _native.stream(dev))
        d['hub_idx'], d['hub_bits'], d['hub_words'] = idx, bits, words

    def _build_edges(self, dev) -> None:
        """edges int32[nnz, 4] (dw_edges_inline_build): {x, deg(x), row_ptr[x] lo, hi}."""
        d = self._dev
        e = torch.empty((max(self.nnz, 1), 4), dtype=torch.int32, device=dev)
        with torch.cuda.device(dev):
            _native.call('dw_edges_inline_build', _native.ptr(d['row_ptr']),
                         _native.ptr(d['col']) if self.nnz else None, self.vocab_size, self.nnz,
                         _native.ptr(e), _native.stream(dev))
        d['edges'] = e

    def _build_adj_hash(self, dev) -> None:
        """adj_off int64[V+1] / adj_hash int32[slots]: dw_adj_hash_offsets + dw_adj_hash_build
        (rows of degree > 8 hashed; the fast node2vec walker's adjacency test in one probe)."""
        import ctypes
        d = self._dev
        V = self.vocab_size
        off = torch.empty(V + 1, dtype=torch.int64, device=dev)
        nbytes = ctypes.c_size_t(0)
        with torch.cuda.device(dev):
            s = _native.stream(dev)
            _native.call('dw_adj_hash_offsets', _native.ptr(d['row_ptr']), V, _native.ptr(off),
                         None, ctypes.byref(nbytes), s)
            tmp = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=dev)
            _native.call('dw_adj_hash_offsets', _native.ptr(d['row_ptr']), V, _native.ptr(off),
                         _native.ptr(tmp), ctypes.byref(nbytes), s)
            n_slots = int(off[V])          # synchronises: the table size
            del tmp
            tab = torch.empty(max(n_slots, 1), dtype=torch.int32, device=dev)
            _native.call('dw_adj_hash_build', _native.ptr(d['row_ptr']),
                         _native.ptr(d['col']) if self.nnz else None, V, _native.ptr(off),
                         n_slots, _native.ptr(tab), _native.ptr(d['status']), s)
        _native.check_status(d['status'], 'adjacency hash build')
        d['adj_off'], d['adj_hash'] = off, tab

    def _sorted_copy(self, dev) -> torch.Tensor:
        d = self._dev
        out = torch.empty(max(self.nnz, 1), dtype=torch.int32, device=dev)
        import ctypes
        nbytes = ctypes.c_size_t(0)
        with torch.cuda.device(dev):
            s = _native.stream(dev)
            _native.call('dw_csr_sort_copy', _native.ptr(d['row_ptr']), _native.ptr(d['col']),
                         self.vocab_size, self.nnz, _native.ptr(out), None, ctypes.byref(nbytes),
                         s)
            tmp = torch.empty(max(int(nbytes.value), 1), dtype=torch.uint8, device=dev)
            _native.call('dw_csr_sort_copy', _native.ptr(d['row_ptr']), _native.ptr(d['col']),
                         self.vocab_size, self.nnz, _native.ptr(out), _native.ptr(tmp),
                         ctypes.byref(nbytes), s)
            del tmp
            # a repeated neighbour in a row (checked once, read by require_simple)
            d['simple_status'] = torch.zeros(1, dtype=torch.int32, device=dev)
            _native.call('dw_csr_check_simple', _native.ptr(d['row_ptr']), _native.ptr(out),
                         self.vocab_size, self.nnz, _native.ptr(d['simple_status']), s)
        return out[:self.nnz] if self.nnz else out

    def require_simple(self, device=None) -> None:
        """Raise ValueError when a row lists the same neighbour twice. The reference walks a
        ``networkx.Graph``, which keeps one entry per neighbour (random_walk_generator.py:41-42);
        the bit-exact node2vec replay relies on that (one position of prev in N(v), class counts
        by intersection), so it refuses such a CSR instead of walking it differently
        (dw_csr_check_simple over col_sorted; one synchronisation per graph and device)."""
        d = self.device_tensors(device, need_sorted=True)
        if d.get('simple_ok'):
            return
        d.pop('simple_ok', None)
        _native.check_status(d['simple_status'], 'CSR check (node2vec replay)')
        d['simple_ok'] = True

    def is_simple(self, device=None) -> bool:
        """require_simple without raising (the Philox walker then keeps the rejection form)."""
        d = self.device_tensors(device, need_sorted=True)
        if 'simple_ok' not in d:
            d['simple_ok'] = int(d['simple_status'].item()) == 0   # one synchronisation
        return bool(d['simple_ok'])

    def _build_alias(self, dev) -> None:
        d = self._dev
        n = max(self.nnz, 1)
        d['prob_thr'] = torch.empty(n, dtype=torch.int32, device=dev)  # uint32 bit pattern
        d['alias'] = torch.empty(n, dtype=torch.int32, device=dev)
        work_p = torch.empty(n, dtype=torch.float64, device=dev)
        work_i = torch.empty(n, dtype=torch.int32, device=dev)
        st = d['status']
        with torch.cuda.device(dev):
            _native.call('dw_alias_build', _native.ptr(d['row_ptr']), _native.ptr(d['weights']),
                         self.vocab_size, self.nnz, _native.ptr(d['prob_thr']),
                         _native.ptr(d['alias']), _native.ptr(work_p), _native.ptr(work_i),
                         _native.ptr(st), _native.stream(dev))
        _native.check_status(st, 'alias build')
