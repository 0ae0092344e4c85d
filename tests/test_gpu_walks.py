"""Walk kernels on the MI355X vs the reference (golden fixtures) and the oracle.

Replay mode: bit-exact integer walks. Fast mode: bit-exact against the Philox restatement
(oracle/philox.py) and statistically against the reference transition law.
"""
import random

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import philox as ph
from oracle import walk_ref

from shallow_encoders.graph.csr import CSRGraph
from shallow_encoders.graph.datasets import GraphTriplets, KarateClubDataset
from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec
from shallow_encoders.graph.rmat import rmat_graph

pytestmark = pytest.mark.gpu

WALK_FIXTURES = ['walks_karate_node2vec_p1_q0.5.npz', 'walks_karate_node2vec_p0.3_q3.npz',
                 'walks_karate_deepwalk.npz', 'walks_triplets_deepwalk.npz',
                 'walks_rmat12_deepwalk.npz', 'walks_rmat12_node2vec_p0.25_q4.npz']


def _csr(f):
    w = f['weights'] if ('weights' in f.files and f['weights'].size) else None
    itos = list(f['itos']) if 'itos' in f.files else None
    return CSRGraph.from_arrays(f['row_ptr'], f['col'], w, itos=itos)


def _walker(f, csr, **kw):
    L = int(f['walk_length'])
    if str(f['method']) == 'node2vec':
        return Node2Vec(csr, L, p=float(f['p']), q=float(f['q']), **kw)
    return DeepWalk(csr, L, **kw)


@pytest.mark.parametrize('name', WALK_FIXTURES)
def test_replay_kernel_bit_exact_vs_reference(name, hip_device):
    f = golden(name)
    csr = _csr(f)
    out = _walker(f, csr).walk_batch(torch.as_tensor(f['starts']), uniforms=f['uniforms'])
    np.testing.assert_array_equal(out.cpu().numpy(), f['walks'])


HUB_FIXTURES = [f'walks_{g}_hubs_{m}.npz' for g in ('rmat16', 'rmat20')
                for m in ('deepwalk', 'node2vec_p0.25_q4', 'node2vec_p1_q1')]


@pytest.mark.parametrize('name', HUB_FIXTURES)
def test_replay_bit_exact_at_hubs_vs_reference(name, hip_device):
    """walks the reference itself took from the top-degree nodes of R-MAT 16 and
    R-MAT 20 (C3's graph: hubs of 44,848 and ~18,500 neighbours), replayed through the default
    path (layout='indexed': DeepWalk over the edge-inline CSR, node2vec's exact picks; no
    DW_REPLAY_SERIAL) — bit-exact. The graph is rebuilt on the device and pinned to the one the
    reference walked by the SHA-256 of its CSR."""
    import hashlib
    import os
    assert os.environ.get('DW_REPLAY_SERIAL', '0') != '1'
    f = golden(name)
    csr = rmat_graph(int(f['scale']), int(f['n_edges']), int(f['graph_seed']), device=hip_device)
    assert hashlib.sha256(np.asarray(csr.row_ptr, dtype='<i8').tobytes()).hexdigest() == \
        str(f['row_ptr_sha256'])
    assert hashlib.sha256(np.asarray(csr.host_col(), dtype='<i4').tobytes()).hexdigest() == \
        str(f['col_sha256'])
    walker = _walker(f, csr, device=hip_device)
    out = walker.walk_batch(torch.as_tensor(f['starts']), uniforms=f['uniforms'])
    np.testing.assert_array_equal(out.cpu().numpy(), f['walks'])
    deg = np.diff(np.asarray(csr.row_ptr))[f['walks'][:, :-1]]
    if int(f['scale']) == 20:   # picks made in rows of >= 10K neighbours, bit-exact
        assert int((deg >= 10_000).sum()) >= 25 and int(deg.max()) == 44_848


@pytest.mark.parametrize('name,cls,kw', [
    ('walks_karate_node2vec_p1_q0.5.npz', KarateClubDataset,
     dict(method='node2vec', method_params={'p': 1, 'q': 0.5})),
    ('walks_karate_node2vec_p0.3_q3.npz', KarateClubDataset,
     dict(method='node2vec', method_params={'p': 0.3, 'q': 3})),
    ('walks_karate_deepwalk.npz', KarateClubDataset, dict(method='deepwalk')),
    ('walks_triplets_deepwalk.npz', GraphTriplets, dict(method='deepwalk'))])
def test_dataset_epoch_end_to_end_bit_exact(name, cls, kw, hip_device):
    """random.seed(s) -> the reference's epoch of walks, through the batched device path."""
    f = golden(name)
    random.seed(int(f['seed']))
    ds = cls(walks_per_node=int(f['walks_per_node']), walk_length=int(f['walk_length']), **kw)
    got = []
    while True:
        b = ds.next_walk_batch(37)
        if b is None:
            break
        got.append(b.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(got), f['walks'])
    np.testing.assert_array_equal(ds._node_ids, f['order_after'])


def test_walk_strings_match_reference(hip_device):
    f = golden('walks_karate_node2vec_p1_q0.5.npz')
    random.seed(int(f['seed']))
    ds = KarateClubDataset(walks_per_node=int(f['walks_per_node']),
                           walk_length=int(f['walk_length']), method='node2vec',
                           method_params={'p': 1, 'q': 0.5})
    itos = list(f['itos'])
    for k, walk in enumerate(ds):
        assert walk == ' '.join(itos[i] for i in f['walks'][k])
        if k == 20:
            break


def _hub_graph(n_leaves=3000, seed=0):
    """A star hub (deg > LDS caps) plus random chords: exercises every replay / staging path."""
    rng = np.random.default_rng(seed)
    n = n_leaves + 1
    edges = [(0, i) for i in range(1, n)]
    chords = set()
    while len(chords) < 4 * n_leaves:
        u, v = rng.integers(1, n, size=2)
        if u != v:
            chords.add((min(u, v), max(u, v)))
    edges += sorted(chords)
    from shallow_encoders.graph.rmat import csr_from_edges
    return csr_from_edges(n, np.asarray(edges, dtype=np.int64))


@pytest.mark.parametrize('method', ['deepwalk', 'node2vec'])
def test_replay_hub_rows_vs_oracle(method, hip_device):
    csr = _hub_graph()
    L = 12
    starts = np.array([2, 3, 4, 1] * 16, dtype=np.int32)  # id 1 = the hub; leaves hit it often
    assert csr.degree()[1] > 2048
    rng = np.random.default_rng(1)
    u = rng.random((len(starts), L - 1))
    w = Node2Vec(csr, L, p=0.5, q=2.0) if method == 'node2vec' else DeepWalk(csr, L)
    got = w.walk_batch(torch.as_tensor(starts), uniforms=u).cpu().numpy()
    g = walk_ref.CSR(csr.row_ptr, csr.col)
    exp = walk_ref.walks_replay(g, starts, L, method, 0.5, 2.0, u)
    np.testing.assert_array_equal(got, exp)
    assert (got == 1).sum() > 16


@pytest.mark.parametrize('layout,L', [('indexed', 16), ('hash', 16), ('csr', 16), ('indexed', 1),
                                      ('indexed', 5), ('indexed', 11), ('hash', 5)])
@pytest.mark.parametrize('method,weighted', [('deepwalk', False), ('deepwalk', True),
                                             ('node2vec', False), ('node2vec', True)])
def test_fast_kernel_bit_exact_vs_philox_oracle(method, weighted, layout, L, hip_device):
    """Fast walkers vs the Philox oracle, every layout; the inline walkers' packed stores at
    walk lengths that are not multiples of 4. Unweighted node2vec on the default layout walks
    over the position index (oracle fast_walks_positions), else by rejection (fast_walks)."""
    f = golden('walks_karate_deepwalk.npz')
    csr = _csr(f) if weighted else CSRGraph.from_arrays(f['row_ptr'], f['col'], None)
    starts = np.arange(1, 35, dtype=np.int32).repeat(3)
    w = (Node2Vec(csr, L, p=0.25, q=4.0, rng='philox', seed=77, layout=layout)
         if method == 'node2vec' else DeepWalk(csr, L, rng='philox', seed=77))
    got = w.walk_batch(torch.as_tensor(starts), walk_id0=1000).cpu().numpy()
    prob, alias = ph.alias_tables(csr.row_ptr, csr.weights) if weighted else (None, None)
    if weighted:
        d = csr.device_tensors(need_alias=True)
        np.testing.assert_array_equal(d['prob_thr'].cpu().numpy().view(np.uint32), prob)
        np.testing.assert_array_equal(d['alias'].cpu().numpy(), alias)
    if method == 'node2vec' and not weighted and layout == 'indexed':
        assert csr.device_tensors().get('n2v_rec') is not None
        exp = ph.fast_walks_positions(csr.row_ptr, csr.col, starts, L, 0.25, 4.0, seed=77,
                                      walk_id0=1000)
    else:
        exp = ph.fast_walks(csr.row_ptr, csr.col, starts, L, method, 0.25, 4.0, seed=77,
                            walk_id0=1000, prob_thr=prob, alias=alias)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize('layout', ['indexed', 'hash', 'csr'])
def test_fast_node2vec_hub_staging_vs_oracle(layout, hip_device):
    """A hub as prev (6-level 8-ary search / a 126-bucket hash row; on the default layout a
    1,500-entry position list); same walks as the oracle."""
    csr = _hub_graph(n_leaves=1500, seed=3)
    L = 8
    starts = np.array([1] * 8 + [6] * 8, dtype=np.int32)   # vocab id 1 is the hub (node 0)
    assert csr.degree()[1] > 1024
    w = Node2Vec(csr, L, p=2.0, q=0.5, rng='philox', seed=5, layout=layout)
    got = w.walk_batch(torch.as_tensor(starts), walk_id0=0).cpu().numpy()
    if layout == 'indexed':
        exp = ph.fast_walks_positions(csr.row_ptr, csr.col, starts, L, 2.0, 0.5, seed=5,
                                      walk_id0=0)
    else:
        exp = ph.fast_walks(csr.row_ptr, csr.col, starts, L, 'node2vec', 2.0, 0.5, seed=5,
                            walk_id0=0)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (4.0, 0.5)])
def test_positions_walkers_int32_lists_vs_oracle(p, q, hip_device):
    """A hub of 66,000 neighbours (> 65,536: its edges' position lists are int32, the rest
    uint16): both position walkers — Philox (dw_walk_fast_positions) and the exact replay
    (dw_walk_replay_positions) — equal their oracles bit for bit on walks through the hub."""
    csr = _hub_graph(n_leaves=66_000, seed=2)
    L = 8
    starts = np.array([1] * 24 + [2, 3, 70, 65_999, 65_500, 40_000, 12, 9] * 3, dtype=np.int32)
    w = Node2Vec(csr, L, p=p, q=q, rng='philox', seed=9)
    got = w.walk_batch(torch.as_tensor(starts), walk_id0=0).cpu().numpy()
    assert csr.device_tensors(hip_device).get('n2v_rec') is not None
    exp = ph.fast_walks_positions(csr.row_ptr, csr.col, starts, L, p, q, seed=9, walk_id0=0)
    np.testing.assert_array_equal(got, exp)
    assert (got[:, 1:] > 65_536).any() and (got == 1).sum() > 24
    u = np.random.default_rng(4).random((len(starts), L - 1))
    got = Node2Vec(csr, L, p=p, q=q, device=hip_device).walk_batch(
        torch.as_tensor(starts), uniforms=u).cpu().numpy()
    ref = walk_ref.walks_replay(walk_ref.CSR(csr.row_ptr, csr.host_col(), None), starts, L,
                                'node2vec', p, q, u)
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0), (0.3, 3.0), (4.0, 0.25)])
def test_fast_positions_walker_vs_oracle_rmat12(p, q, hip_device):
    """The Philox walker over the position index (dw_walk_fast_positions) on the R-MAT-12
    fixture graph (hubs of ~1,000 neighbours, long position lists) from every node, bit-exact
    against oracle/philox.fast_walks_positions; and batch-independent (a walk is a function of
    its walk id)."""
    f = golden('walks_rmat12_node2vec_p0.25_q4.npz')
    csr = CSRGraph.from_arrays(f['row_ptr'], f['col'], None)
    V = csr.vocab_size
    starts = np.arange(1, V, dtype=np.int32)
    starts = starts[np.diff(csr.row_ptr)[1:] > 0][:600]
    L = 12
    w = Node2Vec(csr, L, p=p, q=q, rng='philox', seed=31)
    got = w.walk_batch(torch.as_tensor(starts), walk_id0=5).cpu().numpy()
    exp = ph.fast_walks_positions(csr.row_ptr, csr.col, starts, L, p, q, seed=31, walk_id0=5)
    np.testing.assert_array_equal(got, exp)
    part = w.walk_batch(torch.as_tensor(starts[100:164]), walk_id0=105).cpu().numpy()
    np.testing.assert_array_equal(part, got[100:164])


def _probe_ok(tab, nb, key):
    """Host restatement of the kernel's probe (dw_walk.hip group_hash_contains)."""
    b = ((key * 0x9E3779B1) & 0xFFFFFFFF) * nb >> 32
    for _ in range(nb):
        bk = tab[b * 16:(b + 1) * 16]
        if (bk == key).any():
            return True
        if (bk < 0).any():
            return False
        b = (b + 1) % nb
    return False


@pytest.mark.parametrize('graph', ['rmat12', 'hub'])
def test_adjacency_hash_tables(graph, hip_device):
    """dw_adj_hash_offsets / _build: rows of degree > 8 hold exactly their neighbours in
    ceil(4 deg / 48) buckets; every neighbour is found by the probe and non-neighbours are not."""
    csr = (_csr(golden('walks_rmat12_node2vec_p0.25_q4.npz')) if graph == 'rmat12'
           else _hub_graph(n_leaves=1500, seed=3))
    d = csr.device_tensors(need_adj=True, need_edges=True)
    off = d['adj_off'].cpu().numpy()
    tab = d['adj_hash'].cpu().numpy()
    deg = np.diff(csr.row_ptr)
    nb = np.where(deg > 8, (4 * deg + 47) // 48, 0)
    np.testing.assert_array_equal(np.diff(off), 16 * nb)
    assert off[0] == 0 and (deg > 8).any()
    # edge-inline entries: {x, deg(x), row_ptr[x] as two int32 halves}
    e = d['edges'].cpu().numpy()
    x = csr.col
    np.testing.assert_array_equal(e[:, 0], x)
    np.testing.assert_array_equal(e[:, 1], deg[x])
    np.testing.assert_array_equal(e[:, 2:4].copy().view(np.int64)[:, 0], csr.row_ptr[x])
    rng = np.random.default_rng(0)
    for u in np.flatnonzero(deg > 8):
        t = tab[off[u]:off[u + 1]]
        nbrs = np.sort(csr.col[csr.row_ptr[u]:csr.row_ptr[u + 1]])
        np.testing.assert_array_equal(np.sort(t[t >= 0]), nbrs)
        assert (t >= 0).sum() <= 0.75 * t.size
        for x in nbrs[:: max(1, len(nbrs) // 16)]:
            assert _probe_ok(t, int(nb[u]), int(x))
        others = np.setdiff1d(rng.integers(0, csr.vocab_size, 32), nbrs)
        for x in others:
            assert not _probe_ok(t, int(nb[u]), int(x))


def test_fast_node2vec_statistics_vs_reference_law(hip_device):
    f = golden('walks_karate_node2vec_p0.3_q3.npz')
    csr = _csr(f)
    g = walk_ref.CSR(f['row_ptr'], f['col'], f['weights'])
    prev, v = 1, 3      # n01 -> n03, both high degree with common neighbours
    starts = np.full(200_000, prev, dtype=np.int32)
    w = Node2Vec(csr, 3, p=0.3, q=3.0, rng='philox', seed=11)
    out = w.walk_batch(torch.as_tensor(starts)).cpu().numpy()
    sel = out[out[:, 1] == v][:, 2]
    law = walk_ref.node2vec_transition(g, prev, v, 0.3, 3.0)
    xs = sorted(law)
    counts = np.array([(sel == x).sum() for x in xs], dtype=float)
    expected = np.array([law[x] for x in xs]) * len(sel)
    from scipy.stats import chi2
    stat = ((counts - expected) ** 2 / expected).sum()
    assert len(sel) > 5000
    assert chi2.sf(stat, len(xs) - 1) > 1e-3


def test_isolated_node_raises_like_reference(hip_device):
    import networkx as nx
    g = nx.Graph()
    g.add_edge('a', 'b')
    g.add_node('c')
    w = DeepWalk(g, 4)
    with pytest.raises(IndexError):
        w.walk('c')
    w2 = Node2Vec(g, 4, p=1, q=1, rng='philox')
    with pytest.raises(IndexError):
        w2.walk('c')
    for layout in ('indexed', 'csr'):   # both Philox DeepWalk walkers report it too
        with pytest.raises(IndexError):
            DeepWalk(g, 4, rng='philox', layout=layout).walk('c')
    assert len(DeepWalk(g, 1).walk('c').split()) == 1


def test_fast_walks_rmat20_properties(hip_device):
    """Full benchmark graph: every step is an edge, no aborted walk, deterministic per id."""
    csr = rmat_graph(20, 10_000_000, 0)
    n = 262_144
    starts = torch.arange(1, n + 1, dtype=torch.int32)
    for method in ('deepwalk', 'node2vec'):
        w = (Node2Vec(csr, 80, p=0.25, q=4.0, rng='philox', seed=1) if method == 'node2vec'
             else DeepWalk(csr, 80, rng='philox', seed=1))
        m = n if method == 'deepwalk' else 8192
        out = w.walk_batch(starts[:m], walk_id0=0)
        again = w.walk_batch(starts[:m], walk_id0=0)
        assert torch.equal(out, again)
        # the edge-inline / hash layout == plain CSR + sorted search, at scale (node2vec's
        # default walks over the position index: its own stream, checked below like the rest)
        plain = (Node2Vec(csr, 80, p=0.25, q=4.0, rng='philox', seed=1, layout='csr')
                 if method == 'node2vec' else DeepWalk(csr, 80, rng='philox', seed=1, layout='csr'))
        hashed = (Node2Vec(csr, 80, p=0.25, q=4.0, rng='philox', seed=1, layout='hash')
                  if method == 'node2vec' else w)
        assert torch.equal(hashed.walk_batch(starts[:m], walk_id0=0),
                           plain.walk_batch(starts[:m], walk_id0=0))
        o = out.cpu().numpy()
        assert (o > 0).all()
        sample = o[:: max(1, m // 512)]
        for row in sample:
            for a, b in zip(row[:-1], row[1:]):
                nb = csr.col[csr.row_ptr[a]:csr.row_ptr[a + 1]]
                assert b in nb


@pytest.mark.parametrize('scale,n_edges', [(12, 40_000), (16, 600_000), (20, 10_000_000)])
def test_device_rmat_csr_equals_host_build(hip_device, scale, n_edges):
    """Graph ingestion on the device (dw_rmat_edges -> dw_graph_isolated -> host patch draws
    -> dw_csr_from_edges) reproduces the numpy generator's CSR exactly: same uniforms (numpy
    PCG64 on the device), first-occurrence dedupe, patch edges and networkx row order. At
    scale 20 (C3) it must also give SURVEY.md §8d's check values."""
    import time
    from shallow_encoders.graph.rmat import rmat_edges, rmat_graph
    t0 = time.perf_counter()
    host = rmat_graph(scale, n_edges, 0)
    t1 = time.perf_counter()
    dev = rmat_graph(scale, n_edges, 0, device=hip_device)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'scale {scale}: host {t1 - t0:.2f}s, device {t2 - t1:.2f}s')
    np.testing.assert_array_equal(dev.row_ptr, host.row_ptr)
    np.testing.assert_array_equal(dev.host_col(), host.col)
    assert len(dev.itos) == len(host.itos) and dev.itos[1] == host.itos[1]
    if scale == 20:
        edges, n_patched = rmat_edges(scale, n_edges, 0)
        assert len(edges) == 10_013_665 and n_patched == 475_918
        assert host.nnz == 2 * 10_013_665


def test_node2vec_lane_groups_give_identical_walks(hip_device):
    """The node2vec walker picks 16, 8 or 4 lanes per walker from the batch size (resident
    capacity); walks are pure functions of the walk id, so a walk is the same in every batch."""
    csr = rmat_graph(16, 500_000, 0)
    n_big = 300_000
    starts = (torch.arange(n_big, dtype=torch.int64) % (csr.vocab_size - 1) + 1).to(torch.int32)
    for layout in ('hash', 'csr', 'indexed'):   # ('indexed': the position walker, lane per walk)
        w = Node2Vec(csr, 20, p=0.25, q=4.0, rng='philox', seed=3, layout=layout)
        big = w.walk_batch(starts, walk_id0=0)               # 4 lanes per walker
        mid = w.walk_batch(starts[:40_000], walk_id0=0)      # 8 (or 16) lanes
        small = w.walk_batch(starts[:4096], walk_id0=0)      # 16 lanes
        assert torch.equal(big[:40_000], mid)
        assert torch.equal(big[:4096], small)
        assert (big > 0).all()


def test_cora_epoch_end_to_end_bit_exact(tmp_path, monkeypatch, hip_device):
    """C2's real ingest path: CoraDataset parses the cora.cites / cora.content files the
    reference parsed (synthetic, tests/golden/make_golden.py cora), then random.seed(s) gives
    the reference's epoch of node2vec p=1 q=2 walks through the batched device path."""
    import os
    import shallow_encoders.graph.datasets as ds_mod
    f = golden('walks_cora_node2vec_p1_q2.npz')
    d = tmp_path / 'cora'
    os.makedirs(d)
    (d / 'cora.cites').write_bytes(f['cites_txt'].tobytes())
    (d / 'cora.content').write_bytes(f['content_txt'].tobytes())
    monkeypatch.setattr(ds_mod, 'ASSETS_PATH', str(tmp_path))
    random.seed(int(f['seed']))
    ds = ds_mod.CoraDataset(walks_per_node=int(f['walks_per_node']),
                            walk_length=int(f['walk_length']), method='node2vec',
                            method_params={'p': 1, 'q': 2})
    got = []
    while True:
        b = ds.next_walk_batch(64)
        if b is None:
            break
        got.append(b.cpu().numpy())
    np.testing.assert_array_equal(np.concatenate(got), f['walks'])
    np.testing.assert_array_equal(ds._node_ids, f['order_after'])


def test_counted_node2vec_walks_equal_and_count(hip_device):
    """The counted launches (bench.py's walk roofline): the same walks as the walker, every step
    counted, at least the fixed per-step loads / store counted as bytes — dw_walk_fast_counted
    for the rejection walker (layout 'hash'), dw_walk_fast_positions with counters for the
    default position walker (one 32-B record and a 4-B output per step, 4 B per position
    load, no proposal blocks)."""
    csr = rmat_graph(16, 600_000, 0)
    for layout in ('hash', 'indexed'):
        w = Node2Vec(csr, 20, p=0.25, q=4.0, rng='philox', seed=3, layout=layout)
        for n in (4096, 200_000):                     # 16-lane and 4-lane groups
            starts = (torch.arange(n, dtype=torch.int64) % (csr.vocab_size - 1) + 1).to(
                torch.int32)
            ref = w.walk_batch(starts, walk_id0=5)
            out = torch.empty_like(ref)
            c = w.count_traffic(starts, walk_id0=5, out=out)
            assert torch.equal(out, ref)
            assert c['steps'] == n * 19
            if layout == 'hash':
                assert c['blocks'] >= c['steps'] - n    # >= one proposal block per biased step
                assert c['bytes'] >= c['steps'] * 36 + c['blocks'] * 16
            else:
                assert c['walker'] == 'dw_walk_fast_positions' and c['blocks'] == 0
                assert c['bytes'] == c['steps'] * 36 + 2 * c['position_loads'] + n * 20
                assert c['position_loads'] > 0
                # each search's line moves: at least one per search that loads, at most a
                # move per probe
                assert 0 < c['position_lines'] <= c['position_loads']


@pytest.mark.parametrize('method,p,q,n_walks,L', [('deepwalk', 1.0, 1.0, 65_536, 40),
                                                  ('node2vec', 0.25, 4.0, 1024, 16),
                                                  ('node2vec', 1.0, 1.0, 1024, 16),
                                                  ('node2vec', 0.3, 3.0, 1024, 16)])
def test_replay_exact_picks_equal_serial_replay(method, p, q, n_walks, L, hip_device,
                                                monkeypatch):
    """The replay walker's margin-checked picks (uniform_pick_exact / node2vec_pick_exact, no
    serial sums; their rule is checked against CPython's arithmetic in test_replay_exact.py)
    give bit for bit the walks of the serial replay (DW_REPLAY_SERIAL=1, the path the reference
    fixtures pin) on R-MAT 16 hubs, with uniforms at random and on the step boundaries k/n."""
    csr = rmat_graph(16, 600_000, 0)
    deg = csr.degree()
    starts = torch.as_tensor(np.resize(np.argsort(-deg[1:])[:64] + 1, n_walks).astype(np.int32))
    rng = np.random.default_rng(7)
    u = rng.random((n_walks, L - 1))
    # a quarter of the uniforms exactly on a boundary k/deg of a hub's row (the rule declines)
    u[::4, 0] = (np.arange(len(u[::4])) % (deg[starts.numpy()[::4]] - 1) + 1) / deg[
        starts.numpy()[::4]]
    mk = (lambda: Node2Vec(csr, L, p=p, q=q)) if method == 'node2vec' else (lambda: DeepWalk(csr, L))
    fast = mk().walk_batch(starts, uniforms=u).cpu().numpy()
    # default layout (DeepWalk over the edge-inline CSR, node2vec with hashed adjacency tests)
    # == the plain-CSR replay (layout='csr')
    plain = (Node2Vec(csr, L, p=p, q=q, layout='csr') if method == 'node2vec'
             else DeepWalk(csr, L, layout='csr')).walk_batch(starts, uniforms=u).cpu().numpy()
    np.testing.assert_array_equal(fast, plain)
    monkeypatch.setenv('DW_REPLAY_SERIAL', '1')
    serial = mk().walk_batch(starts, uniforms=u).cpu().numpy()
    np.testing.assert_array_equal(fast, serial)
    assert (fast > 0).all() and int(deg[starts.numpy()].max()) > 2048   # hub rows past LDS


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0), (0.3, 3.0), (2.0, 0.5)])
def test_indexed_node2vec_replay_equals_csr_replay_c3(p, q, hip_device):
    """dw_walk_replay_indexed (default for node2vec, rng='python': the shorter list of each step
    probed through the adjacency hash and its position table) gives bit for bit the walks of
    dw_walk_replay (layout='csr': every neighbour of v classified against sorted N(prev)) on C3's
    graph, from its top hubs and from random nodes; the counted launch gives the same walks."""
    csr = rmat_graph(20, 10_000_000, 0, device=hip_device)
    deg = csr.degree()
    rng = np.random.default_rng(11)
    hubs = np.argsort(-deg[1:])[:256] + 1
    starts = np.concatenate([np.resize(hubs, 2048), rng.integers(1, csr.vocab_size, 2048)])
    starts = torch.as_tensor(starts.astype(np.int32))
    L = 24
    u = torch.from_numpy(rng.random((starts.numel(), L - 1))).to(hip_device)
    idx = Node2Vec(csr, L, p=p, q=q, device=hip_device)
    got = idx.walk_batch(starts, uniforms=u).cpu().numpy()
    ref = Node2Vec(csr, L, p=p, q=q, layout='csr', device=hip_device).walk_batch(
        starts, uniforms=u).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    out = torch.empty((starts.numel(), L), dtype=torch.int32, device=hip_device)
    c = idx.count_replay_traffic(starts, u, out=out)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert c['steps'] == starts.numel() * (L - 1)
    assert c['bytes'] >= c['steps'] * 48 + c['probes'] * 64


def _self_loop_graph():
    # rows with self-loops (t in N(t), v in N(v)), a hub past the hash threshold and short rows
    import networkx as nx
    g = nx.Graph()
    g.add_edges_from([(0, i) for i in range(1, 40)])
    g.add_edges_from([(i, i + 1) for i in range(1, 39)])
    g.add_edges_from([(0, 0), (5, 5), (7, 7), (3, 20), (20, 31)])
    return CSRGraph.from_networkx(nx.relabel_nodes(g, {i: f'n{i}' for i in g.nodes}))


def _self_looped_leaves_graph(n_leaves=300):
    # a hub whose leaves carry self-loops (N(leaf) = {hub, leaf}, some leaves also linked to a
    # neighbour leaf), so a step leaf -> hub has deg(hub) > 64 * deg(leaf): the positions path
    import networkx as nx
    g = nx.Graph()
    g.add_edges_from([('h', f'l{i:03d}') for i in range(n_leaves)])
    g.add_edges_from([(f'l{i:03d}', f'l{i:03d}') for i in range(n_leaves)])
    g.add_edges_from([(f'l{i:03d}', f'l{i + 1:03d}') for i in range(0, n_leaves - 1, 7)])
    g.add_edge('h', 'h')
    return CSRGraph.from_networkx(g)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (2.0, 0.5), (1.0, 1.0)])
def test_node2vec_replay_self_looped_prev_vs_oracle(p, q, hip_device):
    """at a step t -> v where t has a self-loop and deg(v) > 64 * deg(t), the
    positions path mapped t (a member of N(t)) into N(v) as a common neighbour as well as the
    1/p class. The reference gives x == prev only 1/p (random_walk_generator.py:102-104). The
    default walker, the plain-CSR walker and the oracle's restatement agree bit for bit."""
    csr = _self_looped_leaves_graph()
    rng = np.random.default_rng(3)
    leaves = np.arange(2, csr.vocab_size)   # ids: <unk> 0, 'h' 1, leaves after
    starts = torch.as_tensor(rng.choice(leaves, 2048).astype(np.int32))
    L = 12
    u = rng.random((starts.numel(), L - 1))
    got = Node2Vec(csr, L, p=p, q=q, device=hip_device).walk_batch(starts, uniforms=u)
    got = got.cpu().numpy()
    plain = Node2Vec(csr, L, p=p, q=q, layout='csr', device=hip_device).walk_batch(
        starts, uniforms=u).cpu().numpy()
    ref = walk_ref.walks_replay(walk_ref.CSR(csr.row_ptr, csr.host_col(), None),
                                starts.numpy(), L, 'node2vec', p, q, u)
    np.testing.assert_array_equal(plain, ref)
    np.testing.assert_array_equal(got, ref)
    # the path under test was taken: leaf -> hub steps
    assert int((got[:, 1:-1] == 1).sum()) > 1000


def test_node2vec_replay_refuses_repeated_neighbours(hip_device):
    """a CSR row listing a neighbour twice cannot come from the reference's
    nx.Graph, and the exact node2vec picks assume simple rows (one position of prev, class counts
    by intersection): the replay refuses it (dw_csr_check_simple) instead of walking it
    differently from the serial arithmetic; DeepWalk and the Philox walkers take it."""
    # row 1 = {2, 3, 2, 4, ...}: node 2 twice; a hub past the hash threshold elsewhere
    rows = [[], [2, 3, 2, 4], [1, 1, 3], [1, 2], [1] + list(range(5, 20))]
    rows += [[4] for _ in range(5, 20)]
    row_ptr = np.cumsum([0] + [len(r) for r in rows]).astype(np.int64)
    col = np.concatenate([np.asarray(r, dtype=np.int32) for r in rows])
    csr = CSRGraph.from_arrays(row_ptr, col)
    starts = torch.tensor([1, 2, 4], dtype=torch.int32)
    with pytest.raises(ValueError, match='same neighbour twice'):
        Node2Vec(csr, 8, p=0.5, q=2.0, device=hip_device).walk_batch(starts)
    with pytest.raises(ValueError, match='same neighbour twice'):
        Node2Vec(csr, 8, p=0.5, q=2.0, layout='csr', device=hip_device).walk_batch(starts)
    assert DeepWalk(csr, 8, device=hip_device).walk_batch(starts).shape == (3, 8)
    assert Node2Vec(csr, 8, p=0.5, q=2.0, rng='philox',
                    device=hip_device).walk_batch(starts).shape == (3, 8)
    # a simple graph passes the check (karate)
    ok = _csr(golden('walks_karate_node2vec_p1_q0.5.npz'))
    Node2Vec(ok, 4, device=hip_device).walk_batch(torch.tensor([1], dtype=torch.int32))


@pytest.mark.parametrize('which', ['karate', 'rmat12', 'self_loops'])
def test_edge_common_counts_vs_host(which, hip_device):
    """dw_edge_common_counts (the node2vec replay's per-edge class counts: one intersection per
    undirected edge over the shorter list, hub bitmaps or hashes) equals the oracle's
    restatement of the reference rule (walk_ref.edge_class_counts) on every directed edge,
    including self-loops and hub-to-hub edges."""
    if which == 'karate':
        csr = _csr(golden('walks_karate_node2vec_p1_q0.5.npz'))
    elif which == 'rmat12':
        csr = _csr(golden('walks_rmat12_node2vec_p0.25_q4.npz'))
    else:
        csr = _self_loop_graph()
    d = csr.device_tensors(hip_device, need_edge_cn=True)
    got = d['edge_cn'][:csr.nnz].cpu().numpy().view(np.uint32)
    ref = walk_ref.edge_class_counts(walk_ref.CSR(csr.row_ptr, csr.host_col(), None))
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0), (2.0, 0.5)])
def test_node2vec_replay_edge_counts_same_walks(p, q, hip_device, monkeypatch):
    """The replay with the per-edge class counts (a step classifies N(v) from its nearer end up
    to the crossing) gives bit for bit the walks of the whole-row classification, from R-MAT 16's
    hubs and random nodes; the counted launch reads fewer list entries."""
    csr = rmat_graph(16, 600_000, 0, device=hip_device)
    deg = csr.degree()
    rng = np.random.default_rng(5)
    hubs = np.argsort(-deg[1:])[:128] + 1
    starts = torch.as_tensor(np.concatenate([np.resize(hubs, 1024),
                                             rng.integers(1, csr.vocab_size, 1024)]).astype(np.int32))
    L = 40
    u = torch.from_numpy(rng.random((starts.numel(), L - 1))).to(hip_device)
    w = Node2Vec(csr, L, p=p, q=q, device=hip_device)
    monkeypatch.setenv('DW_N2V_EDGE_CN', '0')
    ref = w.walk_batch(starts, uniforms=u).cpu().numpy()
    c0 = w.count_replay_traffic(starts, u)
    monkeypatch.setenv('DW_N2V_EDGE_CN', '1')
    got = w.walk_batch(starts, uniforms=u).cpu().numpy()
    out = torch.empty((starts.numel(), L), dtype=torch.int32, device=hip_device)
    c1 = w.count_replay_traffic(starts, u, out=out)
    np.testing.assert_array_equal(got, ref)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    assert c1['steps'] == c0['steps'] and c1['entries'] < c0['entries']


def _decode_n2v_pos(pos_bytes, boff, cnt, wide):
    """The compact index's lists, flattened in edge order: C(e) uint16 (int32 where wide[e])
    entries at byte boff[e]."""
    out = []
    for e in np.nonzero(cnt)[0]:
        o, c = int(boff[e]), int(cnt[e])
        dt = np.int32 if wide[e] else np.uint16
        out.append(pos_bytes[o:o + c * np.dtype(dt).itemsize].view(dt).astype(np.int64))
    return np.concatenate(out) if out else np.zeros(0, np.int64)


@pytest.mark.parametrize('which', ['karate', 'rmat12', 'self_loops', 'self_looped_leaves',
                                   'hub_66k', 'rmat12_chunked'])
def test_n2v_position_index_vs_oracle(which, hip_device, monkeypatch):
    """dw_n2v_edge_index_build (the node2vec position index: per directed edge t -> v, t's
    position in N(v) and the ascending positions of N(t) ∩ N(v) \\ {t}, uint16 — int32 where
    deg(v) > 65536) equals the oracle's restatement of the reference rule
    (walk_ref.edge_class_positions) on every edge; the 32-B records carry the edge-inline entry,
    the byte offset and the counts word. hub_66k: a hub of 66,000 neighbours (int32 lists);
    rmat12_chunked: the build cut into chunks of 4,096 entries."""
    from shallow_encoders.graph.csr import CSRGraph as _C
    if which == 'rmat12_chunked':
        monkeypatch.setattr(_C, 'N2V_CHUNK_ENTRIES', 4096)
    if which == 'hub_66k':
        csr = _hub_graph(n_leaves=66_000, seed=2)
    elif which == 'karate':
        csr = _csr(golden('walks_karate_node2vec_p1_q0.5.npz'))
    elif which.startswith('rmat12'):
        csr = _csr(golden('walks_rmat12_node2vec_p0.25_q4.npz'))
    elif which == 'self_loops':
        csr = _self_loop_graph()
    else:
        csr = _self_looped_leaves_graph()
    d = csr.device_tensors(hip_device, need_n2v_index=True)
    if which == 'rmat12_chunked':
        assert d['n2v_index_info']['chunks'] > 4
    assert d['n2v_rec'] is not None
    E = csr.nnz
    rec = d['n2v_rec'][:E].cpu().numpy()
    positions = (walk_ref.edge_class_positions_fast if which == 'hub_66k'
                 else walk_ref.edge_class_positions)
    off_ref, pos_ref, pt_ref = positions(walk_ref.CSR(csr.row_ptr, csr.host_col(), None))
    col = csr.host_col()
    rp = np.asarray(csr.row_ptr, dtype=np.int64)
    np.testing.assert_array_equal(rec[:, 0], col)
    np.testing.assert_array_equal(rec[:, 1], rp[col + 1] - rp[col])
    np.testing.assert_array_equal(rec[:, 2].view(np.uint32).astype(np.int64)
                                  | (rec[:, 3].astype(np.int64) << 32), rp[col])
    boff = rec[:, 4].view(np.uint32).astype(np.int64) | (rec[:, 5].astype(np.int64) << 32)
    cnt = np.diff(off_ref)
    wide = (rp[col + 1] - rp[col]) > 65536
    width = np.where(wide, 4, 2)
    boff_ref = np.concatenate([[0], np.cumsum((cnt * width + 3) // 4 * 4)])
    np.testing.assert_array_equal(boff, boff_ref[:-1])
    if which == 'hub_66k':   # (the direct count is O(sum deg^2): from the positions)
        cn = (np.diff(off_ref).astype(np.uint32)
              | np.where(pt_ref >= 0, np.uint32(1 << 31), np.uint32(0)))
    else:
        cn = walk_ref.edge_class_counts(walk_ref.CSR(csr.row_ptr, col, None))
    np.testing.assert_array_equal(rec[:, 6].view(np.uint32), cn)
    np.testing.assert_array_equal(rec[:, 7], pt_ref)
    assert d['n2v_index_info']['entries'] == len(pos_ref)
    assert d['n2v_index_info']['bytes'] == boff_ref[-1] + 32 * E
    if which == 'hub_66k':
        assert wide.sum() == 66_000 and cnt[wide].sum() > 0
    got = _decode_n2v_pos(d['n2v_pos'].cpu().numpy(), boff, cnt, wide)
    np.testing.assert_array_equal(got, pos_ref)


def _boundary_uniforms(csr, starts, L, p, q, rng):
    """Uniforms with a quarter of the walks' first draws exactly on k / deg (the first step's
    margin declines) and a quarter of the second draws on an exact node2vec prefix W_k / T of
    the step the oracle takes there (the position walker's margin declines): those picks are
    made by the serial arithmetic."""
    g = walk_ref.CSR(csr.row_ptr, csr.host_col(), None)
    deg = csr.degree()
    n = len(starts)
    u = rng.random((n, L - 1))
    for w in range(0, n, 4):
        s = int(starts[w])
        u[w, 0] = float(rng.integers(1, deg[s])) / deg[s] if deg[s] > 1 else u[w, 0]
    for w in range(1, n, 4):
        s = int(starts[w])
        v1 = walk_ref.walks_replay(g, np.asarray([s], dtype=np.int32), 2, 'node2vec', p, q,
                                   u[w:w + 1, :1])[0, 1]
        nbrs, wt = walk_ref.node2vec_weights(g, s, int(v1), p, q)
        if len(nbrs) < 2:
            continue
        k = int(rng.integers(0, len(nbrs) - 1))
        u[w, 1] = float(np.sum(wt[:k + 1])) / float(np.sum(wt))
    return u


@pytest.mark.parametrize('which', ['rmat12', 'hub_66k'])
@pytest.mark.parametrize('p,q', [(0.25, 4.0), (2.0, 0.5), (1.0, 1.0), (0.3, 3.0)])
def test_n2v_positions_serial_picks_vs_oracle(p, q, which, hip_device):
    """dw_walk_replay_positions makes a pick its margin cannot decide (uniforms on exact class
    boundaries, at the first step and at a second-order step) by the reference's own fp64
    arithmetic replayed run by run over the position list: the walks equal the oracle's serial
    replay bit for bit (and, on R-MAT 12, the wave walker's, DW_N2V_POS=0), and the counters
    show the serial picks were taken. hub_66k: boundary draws at a 66,000-neighbour hub (its
    int32 lists), non-dyadic 1/p, 1/q included."""
    import os
    rng = np.random.default_rng(17)
    if which == 'rmat12':
        csr = _csr(golden('walks_rmat12_node2vec_p0.25_q4.npz'))
        deg = csr.degree()
        starts = rng.choice(np.nonzero(deg > 0)[0], 512).astype(np.int32)
    else:
        csr = _hub_graph(n_leaves=66_000, seed=2)
        starts = np.concatenate([np.full(24, 1), rng.integers(2, 66_001, 40)]).astype(np.int32)
    L = 12 if which == 'rmat12' else 6
    u = _boundary_uniforms(csr, starts, L, p, q, rng)
    w = Node2Vec(csr, L, p=p, q=q, device=hip_device)
    got = w.walk_batch(torch.as_tensor(starts), uniforms=u).cpu().numpy()
    assert csr.device_tensors(hip_device).get('n2v_rec') is not None
    ref = walk_ref.walks_replay(walk_ref.CSR(csr.row_ptr, csr.host_col(), None), starts, L,
                                'node2vec', p, q, u)
    np.testing.assert_array_equal(got, ref)
    c = w.count_replay_traffic(torch.as_tensor(starts), torch.from_numpy(u).to(hip_device))
    assert c['probes'] > 0, c   # the serial picks
    if which != 'rmat12':
        return
    os.environ['DW_N2V_POS'] = '0'
    try:
        wave = Node2Vec(csr, L, p=p, q=q, device=hip_device).walk_batch(
            torch.as_tensor(starts), uniforms=u).cpu().numpy()
    finally:
        del os.environ['DW_N2V_POS']
    np.testing.assert_array_equal(wave, ref)


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (0.3, 3.0)])
def test_n2v_serial_pick_long_common_list(p, q, hip_device):
    """Twin hubs A, B sharing 70,000 leaves (and the edge A - B): a step B <- A has C = 70,000
    common positions (int32 lists, deg(B) > 65,536). Walks A -> B with the second draw exactly
    on class boundaries of that step: the serial picks run by binades (runs_pass_bs) and equal
    the oracle's replay bit for bit; the walks' other steps too."""
    from shallow_encoders.graph.rmat import csr_from_edges
    n_leaves = 70_000
    A, B = 0, n_leaves + 1
    edges = ([(A, i) for i in range(1, n_leaves + 1)] + [(B, i) for i in range(1, n_leaves + 1)]
             + [(A, B)])
    rng = np.random.default_rng(5)
    chords = rng.integers(1, n_leaves + 1, size=(20_000, 2))
    edges += [(int(a), int(b)) for a, b in chords if a != b]
    edges = sorted({(min(a, b), max(a, b)) for a, b in edges})
    csr = csr_from_edges(n_leaves + 2, np.asarray(edges, dtype=np.int64))
    col = csr.host_col()
    a_id, b_id = A + 1, B + 1                          # vocab ids
    ra = slice(int(csr.row_ptr[a_id]), int(csr.row_ptr[a_id + 1]))
    pos_b = int(np.nonzero(col[ra] == b_id)[0][0])
    deg_a = ra.stop - ra.start
    g = walk_ref.CSR(csr.row_ptr, col, None)
    L, n = 5, 48
    starts = np.full(n, a_id, dtype=np.int32)
    u = rng.random((n, L - 1))
    u[:, 0] = (pos_b + 0.5) / deg_a                     # A -> B
    nbrs, wt = walk_ref.node2vec_weights(g, a_id, b_id, p, q)
    cum = np.cumsum(np.asarray(wt, dtype=np.float64))
    for w in range(n):                                  # B's step on exact class boundaries
        k = int(rng.integers(0, len(nbrs) - 1))
        u[w, 1] = float(np.sum(wt[:k + 1])) / float(np.sum(wt)) if w % 2 == 0 else \
            float(cum[k]) / float(cum[-1])
    wlk = Node2Vec(csr, L, p=p, q=q, device=hip_device)
    got = wlk.walk_batch(torch.as_tensor(starts), uniforms=u).cpu().numpy()
    assert (got[:, 1] == b_id).all()
    ref = walk_ref.walks_replay(g, starts, L, 'node2vec', p, q, u)
    np.testing.assert_array_equal(got, ref)
    c = wlk.count_replay_traffic(torch.as_tensor(starts), torch.from_numpy(u).to(hip_device))
    assert c['probes'] > 0, c


@pytest.mark.parametrize('p,q', [(0.25, 4.0), (1.0, 1.0)])
def test_n2v_positions_equal_wave_walker_c3(p, q, hip_device, monkeypatch):
    """C3's graph (R-MAT 20, hubs of 44,848): the position walker gives the wave walker's walks
    bit for bit from hubs and random nodes, reading a few position entries per step where the
    wave walker reads hundreds of list entries."""
    csr = rmat_graph(20, 10_000_000, 0, device=hip_device)
    deg = csr.degree()
    rng = np.random.default_rng(23)
    hubs = np.argsort(-deg[1:])[:256] + 1
    starts = torch.as_tensor(np.concatenate([np.resize(hubs, 4096),
                                             rng.integers(1, csr.vocab_size, 12288)]
                                            ).astype(np.int32))
    L = 20
    u = torch.from_numpy(rng.random((starts.numel(), L - 1))).to(hip_device)
    w = Node2Vec(csr, L, p=p, q=q, device=hip_device)
    out = torch.empty((starts.numel(), L), dtype=torch.int32, device=hip_device)
    c_pos = w.count_replay_traffic(starts, u, out=out)
    got = out.cpu().numpy()
    assert csr.device_tensors(hip_device)['n2v_rec'] is not None
    monkeypatch.setenv('DW_N2V_POS', '0')
    c_wave = w.count_replay_traffic(starts, u, out=out)
    np.testing.assert_array_equal(got, out.cpu().numpy())
    assert c_pos['steps'] == c_wave['steps'] == starts.numel() * (L - 1)
    assert c_pos['entries'] * 20 < c_wave['entries']
