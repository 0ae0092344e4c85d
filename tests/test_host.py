"""Host-side logic of the product (CPU only): CSR/vocabulary, the replay stream, start-node
order, collate, R-MAT spec, config loading, the C ABI surface, and the fast-mode oracle."""
import os
import random
import re

import numpy as np
import pytest
import torch

from conftest import REPO, golden
from oracle import philox as ph
from oracle import sgns_ref, walk_ref

from shallow_encoders import _native
from shallow_encoders.graph.csr import CSRGraph, node_token
from shallow_encoders.graph.datasets import GraphTriplets, KarateClubDataset, RandomWalkDataset
from shallow_encoders.graph.random_walk_generator import (DeepWalk, Node2Vec,
                                                          random_walk_factory)
from shallow_encoders.graph.rmat import csr_from_edges, rmat_edges
from shallow_encoders.graph.rng import draw_uniforms, skip_uniforms
from shallow_encoders.word2vec.dataloader.torch_dataset import W2VCollateFunctional, tokenize


# ------------------------------------------------------------------------------ CSR / vocab
@pytest.mark.parametrize('name,cls', [('walks_karate_node2vec_p1_q0.5.npz', KarateClubDataset),
                                      ('walks_karate_deepwalk.npz', KarateClubDataset),
                                      ('walks_triplets_deepwalk.npz', GraphTriplets)])
def test_csr_from_networkx_matches_reference_layout(name, cls):
    f = golden(name)
    random.seed(0)
    ds = cls(walks_per_node=1, walk_length=5)
    csr = ds.csr
    assert csr.itos == list(f['itos'])
    np.testing.assert_array_equal(csr.row_ptr, f['row_ptr'])
    np.testing.assert_array_equal(csr.col, f['col'])
    if bool(f['weighted']):
        np.testing.assert_array_equal(csr.weights, f['weights'])
    else:
        assert csr.weights is None


@pytest.mark.parametrize('name', ['walks_rmat12_deepwalk.npz', 'walks_rmat12_node2vec_p0.25_q4.npz'])
def test_rmat_csr_matches_networkx_order(name):
    f = golden(name)
    edges, _ = rmat_edges(int(f['scale']), int(f['n_edges']), int(f['graph_seed']))
    np.testing.assert_array_equal(edges, f['edges'])
    csr = csr_from_edges(1 << int(f['scale']), edges)
    np.testing.assert_array_equal(csr.row_ptr, f['row_ptr'])
    np.testing.assert_array_equal(csr.col, f['col'])


def test_rmat_spec_properties():
    edges, n_patched = rmat_edges(12, 40_000, 0)
    n = 1 << 12
    assert (edges[:, 0] != edges[:, 1]).all()
    key = np.minimum(edges[:, 0], edges[:, 1]) * n + np.maximum(edges[:, 0], edges[:, 1])
    assert len(np.unique(key)) == len(key)
    deg = np.bincount(edges.ravel(), minlength=n)
    assert (deg > 0).all() and n_patched > 0
    g = csr_from_edges(n, edges)
    assert g.vocab_size == n + 1 and g.degree()[0] == 0
    assert g.itos[1] == 'n0000000' and g.itos[-1] == f'n{n - 1:07d}'


def test_node_tokens_and_tokenizer():
    assert node_token('N01') == 'n01'
    assert tokenize('n01 a2 <unk> B7') == ['n01', 'a2', '<unk>', 'b7']
    with pytest.raises(ValueError):
        node_token('12')
    with pytest.raises(ValueError):
        node_token('a b')


# ------------------------------------------------------------------------------ random stream
def test_draw_uniforms_is_the_python_stream():
    random.seed(123)
    a = draw_uniforms(5000)
    after = random.random()
    random.seed(123)
    b = np.array([random.random() for _ in range(5000)])
    np.testing.assert_array_equal(a, b)
    assert random.random() == after
    random.seed(9)
    skip_uniforms(777)
    x = random.random()
    random.seed(9)
    for _ in range(777):
        random.random()
    assert random.random() == x


@pytest.mark.parametrize('name,cls,kw', [
    ('walks_karate_node2vec_p1_q0.5.npz', KarateClubDataset,
     dict(method='node2vec', method_params={'p': 1, 'q': 0.5})),
    ('walks_karate_node2vec_p0.3_q3.npz', KarateClubDataset,
     dict(method='node2vec', method_params={'p': 0.3, 'q': 3})),
    ('walks_karate_deepwalk.npz', KarateClubDataset, dict(method='deepwalk')),
    ('walks_triplets_deepwalk.npz', GraphTriplets, dict(method='deepwalk'))])
def test_dataset_order_and_stream_match_reference(name, cls, kw):
    """Constructor shuffle, the uniforms one epoch consumes, and the end-of-epoch reshuffle."""
    f = golden(name)
    random.seed(int(f['seed']))
    ds = cls(walks_per_node=int(f['walks_per_node']), walk_length=int(f['walk_length']), **kw)
    np.testing.assert_array_equal(ds.start_ids(0, len(ds)), f['starts'])
    np.testing.assert_array_equal(ds._node_ids, f['order'])
    u = draw_uniforms(len(ds) * (int(f['walk_length']) - 1))
    np.testing.assert_array_equal(u.reshape(f['uniforms'].shape), f['uniforms'])
    ds._reshuffle()
    np.testing.assert_array_equal(ds._node_ids, f['order_after'])


def test_factory_contract():
    import networkx as nx
    g = nx.path_graph(['a', 'b', 'c'])
    assert isinstance(random_walk_factory('DeepWalk', g, 3), DeepWalk)
    assert isinstance(random_walk_factory('dfs', g, 3), DeepWalk)
    w = random_walk_factory('node2vec', g, 3, {'p': 2, 'q': 3})
    assert isinstance(w, Node2Vec) and w._params() == (2, 3)
    with pytest.raises(AssertionError):
        random_walk_factory('bfs', g, 3)
    with pytest.raises(TypeError):
        random_walk_factory('deepwalk', g, 3, {'p': 2})
    with pytest.raises(AssertionError):
        DeepWalk(g, 0)
    assert w.get_node_neighbors('b') == ['a', 'c']
    assert w.get_node_normalized_edge_weights('b') == [0.5, 0.5]


def _neumaier_sum(xs):
    """CPython 3.12's float sum() (bltinmodule.c builtin_sum_impl, Neumaier compensation)."""
    s, c = 0.0, 0.0
    for x in xs:
        x = float(x)
        t = s + x
        c += (s - t) + x if abs(s) >= abs(x) else (x - t) + s
        s = t
    return s + c if c else s


def test_replay_on_312_raises_only_where_sums_can_differ(monkeypatch):
    """rng='python' must not refuse the default walkers on CPython >= 3.12. The
    walker raises there only when a step's weight sum could round (3.12 compensates float sums);
    the accepted cases' sums are exact, so naive and compensated summation agree."""
    import networkx as nx
    from shallow_encoders.graph import random_walk_generator as rwg
    g = nx.relabel_nodes(nx.karate_club_graph(), {i: f'n{i + 1:02d}' for i in range(34)})
    gu = nx.Graph(list(g.edges()))                         # the same graph, unweighted
    monkeypatch.setattr(rwg.sys, 'version_info', (3, 12, 0, 'final', 0))
    DeepWalk(gu, 5)                                        # int 1s: always exact
    DeepWalk(g, 5)                                         # integer weights 1-7
    Node2Vec(gu, 5, p=0.25, q=4)                           # 1/p = 4, 1/q = 0.25
    Node2Vec(g, 5, p=1, q=0.5)                             # the karate config
    random_walk_factory('node2vec', gu, 5, {'p': 1, 'q': 1})
    for bad in ({'p': 0.3, 'q': 3}, {'p': 1, 'q': 3}):
        with pytest.raises(NotImplementedError):
            random_walk_factory('node2vec', gu, 5, bad)
    Node2Vec(gu, 5, p=0.3, q=3, rng='philox')              # Philox walkers never sum
    gw = nx.Graph()
    gw.add_edge('a', 'b', weight=0.1)
    gw.add_edge('b', 'c', weight=0.2)
    with pytest.raises(NotImplementedError):
        DeepWalk(gw, 3)
    monkeypatch.setattr(rwg.sys, 'version_info', (3, 10, 12, 'final', 0))
    DeepWalk(gw, 3)                                        # <= 3.11: the serial replay is exact
    # the rule's premise, checked against 3.12's summation: accepted weight sets sum alike
    rng = np.random.default_rng(0)
    for vals in ([1, 4.0, 0.25], [1, 2.0, 1.0], [1.0, 7.0, 3.5, 0.5]):
        for _ in range(200):
            xs = list(rng.choice(vals, size=int(rng.integers(1, 300))))
            assert sum(xs) == _neumaier_sum(xs)
    xs = [1.0, 1.0 / 0.3] * 50 + [1.0 / 3] * 7
    assert sum(xs) != _neumaier_sum(xs)                    # a rejected set: they can differ


# ------------------------------------------------------------------------------ collate
@pytest.mark.parametrize('R', [1, 2, 5])
def test_collate_matches_reference_rule(R):
    rng = np.random.default_rng(R)
    texts = [torch.as_tensor(rng.integers(0, 100, size=rng.integers(2 * R + 1, 40)))
             for _ in range(7)]
    inp, tgt = W2VCollateFunctional('sg', R, 256)(texts)
    ins, tgts = [], []
    for t in texts:
        i, g = sgns_ref.sg_windows(t.numpy()[None, :], R)
        ins.append(i)
        tgts.append(g)
    np.testing.assert_array_equal(inp.numpy(), np.concatenate(ins))
    np.testing.assert_array_equal(tgt.numpy(), np.concatenate(tgts))
    ci, ct = W2VCollateFunctional('cbow', R, 256)(texts)
    np.testing.assert_array_equal(ci.numpy(), tgt.numpy())
    np.testing.assert_array_equal(ct.numpy(), inp.numpy())
    with pytest.raises(AssertionError):
        W2VCollateFunctional('sg', R, 256)([torch.arange(2 * R)])
    clipped, _ = W2VCollateFunctional('sg', R, 2 * R + 3)([torch.arange(50)])
    assert clipped.shape[0] == 3


# ------------------------------------------------------------------------------ configs
@pytest.mark.parametrize('cfg', ['sge_sg_karate_club', 'sge_sg_cora', 'sge_sg_graph_triplets',
                                 'sge_sg_rmat20'])
def test_reference_configs_load(cfg):
    from shallow_encoders.config_parser import load_config
    c = load_config(cfg)
    assert c.datamodule.is_graph and c.datamodule.mode == 'sg'
    assert c.model['_target_'] == 'shallow_encoders.word2vec.model.SkipGram'
    assert c.train.optimizer['_target_'] == 'torch.optim.Adam'
    assert c.analysis.checkpoint == 'last.ckpt'


def test_config_overrides_and_instantiation():
    from shallow_encoders.config_parser import instantiate, load_config
    from shallow_encoders.word2vec.optim import Adam
    c = load_config('sge_sg_cora', overrides=['model.embedding_size=128',
                                              'datamodule.additional_parameters.method_params.q=1'])
    assert c.model['embedding_size'] == 128
    assert c.datamodule.additional_parameters['method_params']['q'] == 1
    m = instantiate(c.model, vocab_size=11)
    assert tuple(m.input_embedding.shape) == (11, 128)
    assert set(m.state_dict()) == {'_input_embedding.weight', '_output_embedding.weight'}
    opt = c.train.instantiate_optimizer(m.parameters())
    assert isinstance(opt, Adam) and opt.param_groups[0]['lr'] == 0.1
    sched = c.train.instantiate_scheduler(opt)
    assert isinstance(sched, torch.optim.lr_scheduler.StepLR)


# ------------------------------------------------------------------------------ C ABI surface
def _header_functions():
    text = open(os.path.join(REPO, 'include', 'dw_hip.h')).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(dw_[a-z0-9_]+)\s*\(', text)))


def test_abi_library_exports_every_declared_symbol():
    lib = _native.load()  # loads without a GPU; no compute call is made
    declared = _header_functions()
    assert declared == sorted(_native.SIGNATURES)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.dw_abi_version() == _native.ABI_VERSION


def test_abi_rejects_bad_arguments_without_a_device():
    lib = _native.load()
    # argument validation returns an error code and sets the message (no launch happens)
    rc = lib.dw_walk_replay(None, None, None, None, 0, None, 1, 0, 0, 1.0, 1.0, None, None, None,
                            None)
    assert rc == _native.DW_E_INVALID_ARG
    assert b'Minimum walk length' in lib.dw_last_error_string()
    rc = lib.dw_sgns_walks(None, 1, 4, 2, 1, 10, 8, None, None, None, None, None, 0, 0, 1.0,
                           None, None, None, 0, None)
    assert rc == _native.DW_E_INVALID_ARG
    assert b'2R+1' in lib.dw_last_error_string()
    import ctypes
    nbytes = ctypes.c_size_t(0)
    rc = lib.dw_sgns_workspace_bytes(573440, 10, 5, 1048577, ctypes.byref(nbytes))
    if torch.cuda.is_available():
        assert rc == 0
        # records (12 B) double-buffered for the sort + hipcub temp storage
        assert nbytes.value >= 573440 * 60 * 24
    else:  # hipcub's temp-size query needs a device; the error is reported, not raised
        assert rc in (0, _native.DW_E_HIP)


def test_product_paths_refuse_host_tensors():
    with pytest.raises(ValueError):
        _native.ptr(torch.zeros(3))


# ------------------------------------------------------------------------------ fast-mode oracle
def test_philox_known_answers():
    # Random123 known-answer vectors for philox4x32-10
    r = ph.philox(0, 0, 0, 0, 0, 0)
    assert [int(x) for x in r] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    m = 0xFFFFFFFF
    r = ph.philox(m, m, m, m, m, m)
    assert [int(x) for x in r] == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    r = ph.philox(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)
    assert [int(x) for x in r] == [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_alias_oracle_represents_the_weights():
    f = golden('walks_karate_deepwalk.npz')
    prob, alias = ph.alias_tables(f['row_ptr'], f['weights'])
    rp = f['row_ptr']
    for r in range(1, len(rp) - 1):
        a, b = rp[r], rp[r + 1]
        n = b - a
        mass = np.zeros(n)
        for i in range(n):
            t = int(prob[a + i])
            pa = 1.0 if t == ph.ALWAYS else t / 4294967296.0
            mass[i] += pa / n
            mass[alias[a + i]] += (1 - pa) / n
        w = f['weights'][a:b]
        np.testing.assert_allclose(mass, w / w.sum(), atol=1e-8)


def test_fast_node2vec_oracle_law_matches_reference_rule():
    """The ballot-rejection restatement samples the reference's transition law."""
    f = golden('walks_karate_node2vec_p0.3_q3.npz')
    g = walk_ref.CSR(f['row_ptr'], f['col'], f['weights'])
    prob, alias = ph.alias_tables(f['row_ptr'], f['weights'])
    # many one-step transitions out of (prev=1, v=34's first neighbour pair) via length-3 walks
    v, prev = 34, int(g.neighbors(34)[0])
    starts = [prev] * 4000
    walks = ph.fast_walks(f['row_ptr'], f['col'], starts, 3, 'node2vec', 0.3, 3.0, seed=5,
                          walk_id0=0, prob_thr=prob, alias=alias)
    sel = walks[walks[:, 1] == v][:, 2]
    law = walk_ref.node2vec_transition(g, prev, v, 0.3, 3.0)
    xs = sorted(law)
    counts = np.array([(sel == x).sum() for x in xs], dtype=float)
    expected = np.array([law[x] for x in xs]) * len(sel)
    chi2 = ((counts - expected) ** 2 / np.maximum(expected, 1e-12)).sum()
    from scipy.stats import chi2 as chi2_dist
    assert len(sel) > 50
    assert chi2_dist.sf(chi2, len(xs) - 1) > 1e-3


def test_device_noise_oracle_is_uniform():
    nz = ph.device_noise(seed=3, noise_offset=0, n_centres=400, n_ctx=4, k=5, vocab_size=7)
    assert nz.shape == (400, 4, 5) and nz.min() >= 0 and nz.max() < 7
    counts = np.bincount(nz.ravel(), minlength=7)
    from scipy.stats import chisquare
    assert chisquare(counts).pvalue > 1e-3


@pytest.mark.parametrize('n,seed', [(4096, 0), (65_537, 1), (131_072, 2), (1_000_003, 3)])
def test_native_shuffle_matches_cpython(n, seed):
    """dw_host_shuffle (the start-node shuffle in native code) == random.shuffle bit for bit, and
    the global stream continues where Python's own shuffle leaves it."""
    import random
    from shallow_encoders.graph.rng import shuffled_range
    random.seed(seed)
    random.random()                       # an arbitrary position inside the 624-word block
    ref = list(range(n))
    random.shuffle(ref)
    after_ref = [random.random() for _ in range(5)]
    random.seed(seed)
    random.random()
    got = shuffled_range(n)
    after_got = [random.random() for _ in range(5)]
    assert np.array_equal(got, np.asarray(ref, dtype=np.int64))
    assert after_got == after_ref


def _cora_assets(f, root):
    d = os.path.join(root, 'cora')
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, 'cora.cites'), 'wb') as fh:
        fh.write(f['cites_txt'].tobytes())
    with open(os.path.join(d, 'cora.content'), 'wb') as fh:
        fh.write(f['content_txt'].tobytes())
    return root


def test_cora_ingest_matches_reference(tmp_path, monkeypatch):
    """C2's ingest path: CoraDataset (datasets.py:183-221) on the synthetic cora.cites /
    cora.content the reference itself parsed (tests/golden/make_golden.py cora): the same graph,
    vocabulary, CSR in networkx neighbour order, start-node order, labels and features."""
    import shallow_encoders.graph.datasets as ds_mod
    f = golden('walks_cora_node2vec_p1_q2.npz')
    monkeypatch.setattr(ds_mod, 'ASSETS_PATH', _cora_assets(f, str(tmp_path)))
    random.seed(int(f['seed']))
    ds = ds_mod.CoraDataset(walks_per_node=int(f['walks_per_node']),
                            walk_length=int(f['walk_length']), method='node2vec',
                            method_params={'p': 1, 'q': 2})
    assert ds.graph.number_of_nodes() == int(f['n_nodes'])
    assert ds.graph.number_of_edges() == int(f['n_edges'])
    assert list(ds.csr.itos) == list(f['itos'])
    np.testing.assert_array_equal(ds.csr.row_ptr, f['row_ptr'])
    np.testing.assert_array_equal(ds.csr.col, f['col'])
    np.testing.assert_array_equal(ds._node_ids, f['order'])
    names = list(f['label_names'])
    assert sorted(ds.labels) == names
    assert [ds.labels[n] for n in names] == list(f['label_values'])
    np.testing.assert_array_equal(np.stack([ds.features[n] for n in names[:16]]),
                                  f['feature_sample'])


def test_step_scalars_layout_and_history():
    """word2vec/graphed.py's dw_step_scalars block matches include/dw_hip.h's struct (56 bytes,
    walk_id0 @0, noise_offset @8, step @16, adam[8] @24) and its Adam history rows equal the
    scalars the eager launches pass (adam_scalars rounded to float32, then the reciprocal)."""
    import ctypes
    from shallow_encoders.word2vec.graphed import _STEP_DTYPE, adam_history
    from shallow_encoders.word2vec.sharding import adam_scalars

    class StepScalars(ctypes.Structure):
        _fields_ = [('walk_id0', ctypes.c_uint64), ('noise_offset', ctypes.c_uint64),
                    ('step', ctypes.c_int64), ('adam', ctypes.c_float * 8)]
    assert ctypes.sizeof(StepScalars) == _STEP_DTYPE.itemsize == 56
    for name in ('walk_id0', 'noise_offset', 'step', 'adam'):
        assert getattr(StepScalars, name).offset == _STEP_DTYPE.fields[name][1]
    header = open(os.path.join(REPO, 'include', 'dw_hip.h')).read()
    body = header[header.index('typedef struct dw_step_scalars'):]
    body = body[:body.index('} dw_step_scalars;')]
    assert re.findall(r'(uint64_t|int64_t|float) (\w+)', body) == [
        ('uint64_t', 'walk_id0'), ('uint64_t', 'noise_offset'), ('int64_t', 'step'),
        ('float', 'adam')]
    h = adam_history(5, 0.01, (0.9, 0.999), 1e-8, 0.0)
    for s in range(1, 6):
        exp = [ctypes.c_float(x).value for x in adam_scalars(s, 0.01, (0.9, 0.999), 1e-8, 0.0)]
        # [7]: the correctly rounded fp32 reciprocal of sqrt(bias_correction2) (dw::div_bc2s)
        assert h[s, :7].tolist() == exp and h[s, 7] == np.float32(1.0) / np.float32(exp[3])


# ------------------------------------------------------------------------------ MT19937 stream
def _py_state(seed, skip):
    r = random.Random(seed)
    for _ in range(skip):
        r.random()
    st = r.getstate()[1]
    return r, list(st[:624]), st[624]


@pytest.mark.parametrize('seed,skip', [(0, 0), (7, 1), (11, 311), (13, 312), (5, 1000)])
def test_mt_oracle_stream_is_cpython_random(seed, skip):
    """oracle/mt_ref.py's raw-sequence restatement gives random.random() and the state after."""
    from oracle import mt_ref
    r, mt, idx = _py_state(seed, skip)
    n = 2000
    out, arr, index = mt_ref.stream(mt, idx, n)
    exp = np.array([r.random() for _ in range(n)])
    np.testing.assert_array_equal(out, exp)
    st = r.getstate()[1]
    assert list(arr) == list(st[:624]) and index == st[624]


def test_mt_characteristic_polynomial_annihilates_the_stream():
    """phi (135 terms, degree 19937) kills every bit plane of the raw sequence, so t^J mod phi
    gives the jump (Cayley-Hamilton on the 19937-bit state)."""
    from oracle import mt_ref
    _, mt, _ = _py_state(3, 17)
    x = mt_ref.raw_sequence(mt, 60_000)
    assert len(mt_ref.PHI_TERMS) == 134
    assert mt_ref.annihilates(x, range(0, 60_000 - 19_938, 997))
    assert not mt_ref.annihilates(x ^ np.uint32(1) * (np.arange(x.size) == 20_000), [20_000])


def test_mt_jump_table_matches_restatement_and_jumps():
    """dw_mt_jump_table (host C ABI) = the exponents of t^(624 S c - 2) mod phi computed in
    Python; applied to the raw sequence they give x[J + 1 .. J + 625]."""
    from oracle import mt_ref
    from shallow_encoders import _native
    _native.load()
    _, mt, _ = _py_state(21, 5)
    for stride, chains in ((1, 5), (3, 3), (256, 3)):
        off = np.zeros(chains + 1, dtype=np.int64)
        pos = np.zeros(chains * 19937, dtype=np.uint16)
        _native.call('dw_mt_jump_table', stride, chains, off.ctypes.data, pos.ctypes.data,
                     pos.size)
        assert off[0] == off[1] == 0
        x = mt_ref.raw_sequence(mt, 624 * stride * chains + 20_600)
        base = x[:19937 + 626]
        for c in range(1, chains):
            J = 624 * stride * c - 2
            ls = pos[off[c]:off[c + 1]].astype(np.int64)
            if stride == 256 and c == 1:
                np.testing.assert_array_equal(ls, mt_ref.exponents(mt_ref.t_pow_mod(J)))
            got = mt_ref.jump(base, ls, np.arange(1, 626))
            np.testing.assert_array_equal(got, x[J + 1:J + 626])
    with pytest.raises(_native.DWError):
        _native.call('dw_mt_jump_table', 256, 3, off.ctypes.data, pos.ctypes.data, 100)


@pytest.mark.parametrize('stride,seed,skip,n', [(1, 1, 0, 1500), (1, 2, 1, 1500),
                                                (2, 3, 311, 4001), (3, 4, 312, 2),
                                                (1, 5, 623, 937)])
def test_mt_chained_generation_is_cpython_random(stride, seed, skip, n):
    """dw_mt_uniforms' decomposition (chains of `stride` windows seeded by the product's jump
    table; doubles whose words straddle windows and chains; the final state) restated in numpy,
    against CPython — odd and even start indices, a draw from the state's last word."""
    from oracle import mt_ref
    from shallow_encoders import _native
    _native.load()
    r, mt, idx = _py_state(seed, skip)
    windows = (idx + 2 * n - 1) // 624 + 1
    chains = -(-windows // stride)
    off = np.zeros(chains + 1, dtype=np.int64)
    pos = np.zeros(chains * 19937, dtype=np.uint16)
    _native.call('dw_mt_jump_table', stride, chains, off.ctypes.data, pos.ctypes.data, pos.size)
    out, arr, index = mt_ref.uniforms_chained(mt, idx, n, stride, pos, off)
    np.testing.assert_array_equal(out, np.array([r.random() for _ in range(n)]))
    st = r.getstate()[1]
    assert list(arr) == list(st[:624]) and index == st[624]


@pytest.mark.parametrize('seed,skip,high,n', [(0, 0, 2708, 3000), (1234, 5, 1_048_577, 700),
                                              (7, 623, 34, 1), (99, 624, 2 ** 32 - 1, 2000),
                                              (3, 400, 5, 0), (8, 1, 2 ** 28 - 1, 999),
                                              (9, 2, 2 ** 28, 999), (10, 311, 2 ** 30 + 3, 313)])
def test_torch_randint_oracle_and_state_mapping(seed, skip, high, n):
    """The reference's negatives are torch.randint on torch's CPU generator
    (utils/sampling.py:7-21). oracle.mt_ref.torch_randint restates it from the MT19937 state in
    CPython's layout, and graph/rng.py maps torch.get_rng_state() onto that layout and back
    (_torch_state_words / _torch_state_with): the values and the generator state after them equal
    torch's own, for fresh seeds (index 624), odd positions and a window's last word."""
    from oracle import mt_ref
    from shallow_encoders.graph.rng import _torch_state_with, _torch_state_words
    torch.manual_seed(seed)
    if skip:
        torch.randint(0, 3, (skip,))
    st0 = torch.get_rng_state()
    words, index = _torch_state_words(st0)
    vals, arr, idx = mt_ref.torch_randint(words, index, n, high)
    exp = torch.randint(0, high, (n,), dtype=torch.long).numpy()
    np.testing.assert_array_equal(vals, exp)
    assert torch.equal(_torch_state_with(st0, arr, idx), torch.get_rng_state())
    # the mapping round-trips (a fresh seed's next = 0 is written as 624: the same position)
    torch.set_rng_state(_torch_state_with(st0, words, index))
    after = torch.randint(0, high, (n + 5,), dtype=torch.long)
    torch.set_rng_state(st0)
    assert torch.equal(after, torch.randint(0, high, (n + 5,), dtype=torch.long))


def test_library_built_from_these_sources():
    """The shipped libdw_hip.so carries the hash of the sources it was built from
    (csrc/build.py source_id, dw_build_id()): equal to this tree's, so the binary that travels
    to the GPU box is not stale."""
    import importlib.util
    from shallow_encoders import _native
    spec = importlib.util.spec_from_file_location(
        'dw_build', os.path.join(os.path.dirname(_native.__file__), '..', 'csrc', 'build.py'))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    assert _native.load().dw_build_id().decode() == b.source_id()


def test_hist_box_header():
    """Row 0 of a lazy Adam history (include/dw_hip.h DW_HIST_BOX_TAG): the tag and the first
    step from which every written row keeps the g = 0 replays in the box (dw::replay_g0's
    unscaled sqrt / division). The tests are dw::in_bits' on the float32 bits."""
    from shallow_encoders.word2vec.sharding import (HIST_BOX_TAG, hist_header, hist_row,
                                                    hist_rows_in_box)
    def hist(n, wd_at=(), eps=1e-8, betas=(0.9, 0.999)):
        h = np.zeros((n + 1, 8), dtype=np.float32)
        for s in range(1, n + 1):
            h[s] = hist_row(s, 0.01, betas, eps, 0.01 if s in wd_at else 0.0)
        return h
    h = hist(20)
    h0 = hist_header(h, 20)
    assert h0.view(np.uint32)[0] == HIST_BOX_TAG == 0x58424457 and h0.view(np.int32)[1] == 1
    # [4], [5]: the box rows' constant 1 - beta1 and beta2 (the frozen replay tails use them)
    assert h0[4] == h[1, 0] and h0[5] == h[1, 1]
    hv = hist(20)
    hv[12:] = np.stack([hist_row(s, 0.01, (0.8, 0.999), 1e-8, 0.0) for s in range(12, 21)])
    hv0 = hist_header(hv, 20)
    assert np.isnan(hv0[4]) and np.isnan(hv0[5])
    assert hist_header(hist(20, wd_at=(3, 7)), 20).view(np.int32)[1] == 8
    assert hist_header(hist(20, wd_at=(20,)), 20).view(np.int32)[1] == 21
    assert hist_header(hist(20, eps=1e-9), 20).view(np.int32)[1] == 21     # eps < 2^-27
    assert hist_rows_in_box(hist(3, eps=2.0 ** -27)[1:]).all()
    assert not hist_rows_in_box(hist(3, eps=1.5)[1:]).any()
    # sqrt(bias_correction2) < 2^-10 (beta2 = 1 - 1e-7 at step 1): out; later steps in
    hb = hist(40, betas=(0.9, 1 - 1e-7))
    assert not hist_rows_in_box(hb[1:2]).any()
    r = hb.copy()
    r[:, 6] = -0.0                                                            # -0 is not +0
    assert not hist_rows_in_box(r[1:]).any()
    r = h.copy()
    r[:, 7] = 0.0                                                             # no reciprocal
    assert not hist_rows_in_box(r[1:]).any()
    r = h.copy()
    r[:, 0] = -0.1                                                            # a sign bit fails
    assert not hist_rows_in_box(r[1:]).any()
