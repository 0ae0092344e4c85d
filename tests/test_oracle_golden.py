"""The oracle against the reference's own outputs (golden fixtures). CPU only.

Pins oracle/walk_ref.py and oracle/sgns_ref.py before any device result is judged by them.
"""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle import sgns_ref, walk_ref

# (the hub fixtures store the graph's spec and digest instead of its CSR: tested below)
WALK_FIXTURES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, 'walks_*.npz'))
                       if '_hubs_' not in p)
SGNS_FIXTURES = sorted(os.path.basename(p) for p in glob.glob(os.path.join(GOLDEN, 'sgns_*.npz')))


def _graph(f):
    w = f['weights'] if ('weights' in f.files and f['weights'].size) else None
    return walk_ref.CSR(f['row_ptr'], f['col'], w)


@pytest.mark.parametrize('name', WALK_FIXTURES)
def test_oracle_replays_reference_walks_bit_exact(name):
    f = golden(name)
    g = _graph(f)
    out = walk_ref.walks_replay(g, f['starts'], int(f['walk_length']), str(f['method']),
                                float(f['p']), float(f['q']), f['uniforms'])
    np.testing.assert_array_equal(out, f['walks'])


@pytest.mark.parametrize('name', [n for n in WALK_FIXTURES if 'karate' in n or 'triplets' in n])
def test_oracle_transition_law_matches_reference(name):
    """Every random.choices weight vector the reference used equals the oracle's law."""
    f = golden(name)
    g = _graph(f)
    walks, L = f['walks'], int(f['walk_length'])
    offs, pop, w = f['step_off'], f['step_pop'], f['step_w']
    method, p, q = str(f['method']), float(f['p']), float(f['q'])
    k = 0
    for wk in walks:
        prev = None
        for s in range(1, L):
            v = int(wk[s - 1])
            a, b = offs[k], offs[k + 1]
            law = walk_ref.node2vec_transition(g, prev if method == 'node2vec' else None, v,
                                               p if method == 'node2vec' else 1.0,
                                               q if method == 'node2vec' else 1.0)
            np.testing.assert_array_equal(pop[a:b], g.neighbors(v))
            got = np.array([law[x] for x in pop[a:b]])
            np.testing.assert_array_equal(got, w[a:b])  # bit-exact normalised weights
            prev = v
            k += 1
    assert k == len(offs) - 1


def _max_norm(f):
    if 'max_norm' not in f.files or np.isnan(float(f['max_norm'])):
        return None
    return float(f['max_norm'])


@pytest.mark.parametrize('name', SGNS_FIXTURES)
def test_oracle_sgns_matches_reference(name):
    f = golden(name)
    mn = _max_norm(f)
    loss, g_in, g_out, rec, prec, w_in_r, w_out_r = sgns_ref.sgns_forward_backward(
        f['w_in0'], f['w_out0'], f['inputs'], f['targets'], f['noise'][0], max_norm=mn,
        return_tables=True)
    if 'w_in0r' in f.files:   # the tables the reference's forwards renormalised (max_norm)
        np.testing.assert_array_equal(w_in_r, f['w_in0r'])
        np.testing.assert_array_equal(w_out_r, f['w_out0r'])
    np.testing.assert_allclose([loss['loss'], loss['positive-loss'], loss['negative-loss']],
                               f['losses'][0], rtol=1e-6)
    np.testing.assert_allclose(g_in, f['g_in'], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(g_out, f['g_out'], rtol=1e-5, atol=1e-9)
    assert rec == pytest.approx(float(f['recall'][0]))
    assert prec == pytest.approx(float(f['precision'][0]))
    if f['inputs'].reshape(len(f['targets']), -1).shape[1] != 1:
        return   # the closed form below is the skip-gram one
    # independent float64 closed form of the same gradient (clamp mask + batch mean)
    l64, gi64, go64 = sgns_ref.sgns_grads_closed_form(w_in_r, w_out_r, f['inputs'],
                                                      f['targets'], f['noise'][0])
    assert l64 == pytest.approx(float(f['losses'][0][0]), rel=1e-5)
    np.testing.assert_allclose(gi64, f['g_in'], rtol=1e-4, atol=1e-8)
    np.testing.assert_allclose(go64, f['g_out'], rtol=1e-4, atol=1e-8)


@pytest.mark.parametrize('name', SGNS_FIXTURES)
def test_oracle_adam_trajectory_matches_reference(name):
    f = golden(name)
    ref = sgns_ref.TorchAdamRef(f['w_in0'], f['w_out0'], lr=float(f['lr']))
    for step in range(f['noise'].shape[0]):
        loss = ref.train_step(f['inputs'], f['targets'], f['noise'][step], max_norm=_max_norm(f))
        assert loss['loss'] == pytest.approx(float(f['losses'][step][0]), rel=1e-6)
        if step == 0:
            w_in, w_out = ref.tables()
            np.testing.assert_allclose(w_in, f['w_in1'], rtol=1e-6, atol=1e-7)
            np.testing.assert_allclose(w_out, f['w_out1'], rtol=1e-6, atol=1e-7)
    w_in, w_out = ref.tables()
    np.testing.assert_allclose(w_in, f['w_in_n'], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(w_out, f['w_out_n'], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize('name', SGNS_FIXTURES)
def test_oracle_windows_match_reference_collate(name):
    f = golden(name)
    cbow = 'mode' in f.files and str(f['mode']) == 'cbow'
    ins, tgt = (sgns_ref.cbow_windows if cbow else sgns_ref.sg_windows)(f['walks'], int(f['R']))
    np.testing.assert_array_equal(ins, f['inputs'])
    np.testing.assert_array_equal(tgt, f['targets'])


def test_oracle_trajectory_with_steplr():
    import torch
    f = golden('traj_karate_node2vec.npz')
    ref = sgns_ref.TorchAdamRef(f['w_in0'], f['w_out0'], lr=float(f['lr']))
    sched = torch.optim.lr_scheduler.StepLR(ref.opt, step_size=int(f['step_size']),
                                            gamma=float(f['gamma']))
    R, K = int(f['R']), int(f['K'])
    offs = np.concatenate([[0], np.cumsum(f['batch_sizes'])])
    noff = 0
    epoch = 0
    for step, nb in enumerate(f['batch_sizes']):
        if f['epoch_of_step'][step] != epoch:
            sched.step()
            epoch = int(f['epoch_of_step'][step])
        walks = f['walks'][offs[step]:offs[step + 1]]
        ins, tgt = sgns_ref.sg_windows(walks, R)
        nz = f['noise'][noff:noff + len(ins)]
        noff += len(ins)
        assert ref.opt.param_groups[0]['lr'] == pytest.approx(float(f['lrs'][step]))
        loss = ref.train_step(ins, tgt, nz)
        assert loss['loss'] == pytest.approx(float(f['losses'][step]), rel=1e-6)
    w_in, w_out = ref.tables()
    np.testing.assert_allclose(w_in, f['w_in'], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(w_out, f['w_out'], rtol=1e-5, atol=1e-6)


# ---- the vectorised / torch forms the full-size checks use, against the definitions ----------

def test_bounded64_vectorised_equals_integer_definition():
    from oracle import philox as ph
    rng = np.random.default_rng(3)
    lo = np.concatenate([rng.integers(0, 2 ** 32, 4000, dtype=np.uint64),
                         np.array([0, 2 ** 32 - 1, 0, 2 ** 32 - 1], np.uint64)])
    hi = np.concatenate([rng.integers(0, 2 ** 32, 4000, dtype=np.uint64),
                         np.array([0, 0, 2 ** 32 - 1, 2 ** 32 - 1], np.uint64)])
    for n in (1, 35, 1_048_577, 16_777_217, 2 ** 31 - 1, 2 ** 32 - 1):
        exp = ph.bounded64_int(lo, hi, n)
        np.testing.assert_array_equal(ph.bounded64(lo, hi, n), exp)
        if n < 2 ** 31:
            import torch
            got = ph.bounded64_torch(torch.as_tensor(lo.astype(np.int64)),
                                     torch.as_tensor(hi.astype(np.int64)), n)
            np.testing.assert_array_equal(got.numpy(), exp)


def test_philox_torch_equals_numpy_and_device_noise_torch():
    import torch
    from oracle import philox as ph
    rng = np.random.default_rng(4)
    c = [rng.integers(0, 2 ** 32, 500, dtype=np.uint64) for _ in range(4)]
    exp = ph.philox(*c, 0x12345678, 0x9ABCDEF0)
    got = ph.philox_torch(*(torch.as_tensor(x.astype(np.int64)) for x in c),
                          0x12345678, 0x9ABCDEF0)
    for e, g in zip(exp, got):
        np.testing.assert_array_equal(g.numpy().astype(np.uint64), e)
    for (B, C, K, V, off) in ((37, 10, 5, 1_048_577, 123_456_789_012), (9, 4, 3, 35, 0),
                              (5, 2, 1, 2 ** 31 - 1, 7)):
        np.testing.assert_array_equal(ph.device_noise_torch(99, off, B, C, K, V).numpy(),
                                      ph.device_noise(99, off, B, C, K, V))


def test_closed_form_torch_and_windows_torch_equal_numpy_forms():
    import torch
    f = golden('sgns_d128_k5.npz')
    R = int(f['R'])
    ins_t, tgt_t = sgns_ref.sg_windows_torch(torch.as_tensor(f['walks']), R)
    ins, tgt = sgns_ref.sg_windows(f['walks'], R)
    np.testing.assert_array_equal(ins_t.numpy(), ins.reshape(-1))
    np.testing.assert_array_equal(tgt_t.numpy(), tgt)
    l64, gi64, go64 = sgns_ref.sgns_grads_closed_form(f['w_in0'], f['w_out0'], ins, tgt,
                                                      f['noise'][0])
    sums, gi, go = sgns_ref.sgns_grads_closed_form_torch(
        torch.as_tensor(f['w_in0']), torch.as_tensor(f['w_out0']), ins_t, tgt_t,
        torch.as_tensor(f['noise'][0]), chunk=7)
    assert float(sums[0] + sums[1]) / tgt.size == pytest.approx(l64, rel=1e-12)
    np.testing.assert_allclose(gi.numpy(), gi64, rtol=1e-12, atol=1e-18)
    np.testing.assert_allclose(go.numpy(), go64, rtol=1e-12, atol=1e-18)
    assert float(sums[0] + sums[1]) / tgt.size == pytest.approx(float(f['losses'][0][0]),
                                                                rel=1e-5)


@pytest.mark.parametrize('m', ['deepwalk', 'node2vec_p0.25_q4', 'node2vec_p1_q1'])
def test_oracle_replays_reference_hub_walks_rmat16(m):
    """The oracle walker against the reference's walks from R-MAT 16's top hubs (the graph
    rebuilt on the host and pinned by its CSR digest; tests/golden/make_golden.py hubs)."""
    import hashlib
    from shallow_encoders.graph.rmat import rmat_graph
    f = golden(f'walks_rmat16_hubs_{m}.npz')
    csr = rmat_graph(int(f['scale']), int(f['n_edges']), int(f['graph_seed']))
    assert hashlib.sha256(np.asarray(csr.row_ptr, dtype='<i8').tobytes()).hexdigest() == \
        str(f['row_ptr_sha256'])
    assert hashlib.sha256(np.asarray(csr.col, dtype='<i4').tobytes()).hexdigest() == \
        str(f['col_sha256'])
    g = walk_ref.CSR(csr.row_ptr, csr.col, None)
    out = walk_ref.walks_replay(g, f['starts'], int(f['walk_length']), str(f['method']),
                                float(f['p']), float(f['q']), f['uniforms'])
    np.testing.assert_array_equal(out, f['walks'])
    # the numpy-backed undirected form (test_gpu_c5_walks' oracle at R-MAT 24) on the same
    # reference walks
    ga = walk_ref.ArrayCSR(csr.row_ptr, csr.col, None, undirected=True)
    out = walk_ref.walks_replay(ga, f['starts'], int(f['walk_length']), str(f['method']),
                                float(f['p']), float(f['q']), f['uniforms'])
    np.testing.assert_array_equal(out, f['walks'])


def test_column_chunked_closed_form_equals_numpy_form():
    """sgns_coefs_torch + sgns_grad_columns_torch (the C5 full-scale test's reference: tables
    too large for a float64 copy) equal the numpy closed form, column slab by column slab,
    with the in-table gradient compacted to the touched rows."""
    import torch
    f = golden('sgns_d256_k5_r5.npz')
    R = int(f['R'])
    ins_t, tgt_t = sgns_ref.sg_windows_torch(torch.as_tensor(f['walks']), R)
    ins, tgt = sgns_ref.sg_windows(f['walks'], R)
    l64, gi64, go64 = sgns_ref.sgns_grads_closed_form(f['w_in0'], f['w_out0'], ins, tgt,
                                                      f['noise'][0])
    w_in, w_out = torch.as_tensor(f['w_in0']), torch.as_tensor(f['w_out0'])
    noise = torch.as_tensor(f['noise'][0])
    sums, ds, dt, _ = sgns_ref.sgns_coefs_torch(w_in, w_out, ins_t, tgt_t, noise, chunk=5)
    assert float(sums[0] + sums[1]) / tgt.size == pytest.approx(l64, rel=1e-12)
    rows = torch.unique(ins_t)
    index = torch.full((w_in.shape[0],), -1, dtype=torch.int64)
    index[rows] = torch.arange(rows.numel())
    d = w_in.shape[1]
    for c0 in range(0, d, 96):
        c1 = min(d, c0 + 96)
        gi, go = sgns_ref.sgns_grad_columns_torch(w_in, w_out, ins_t, tgt_t, noise, ds, dt, c0,
                                                  c1, index, rows.numel(), chunk=9)
        np.testing.assert_allclose(gi.numpy(), gi64[rows.numpy(), c0:c1], rtol=1e-12,
                                   atol=1e-18)
        np.testing.assert_allclose(go.numpy(), go64[:, c0:c1], rtol=1e-12, atol=1e-18)
    untouched = np.setdiff1d(np.arange(w_in.shape[0]), rows.numpy())
    assert not gi64[untouched].any()


def test_oracle_d128_trajectory_matches_reference():
    """24 reference Adam steps at d=128, K=5, R=5, lr 0.01 (traj_d128_k5_r5.npz): the oracle
    replays the losses and final tables, and the fixture's negatives are torch's global stream
    after manual_seed(noise_seed) (what Word2VecTrainer(noise='torch') draws)."""
    import torch
    from shallow_encoders.word2vec.utils.sampling import generate_noise_batch
    f = golden('traj_d128_k5_r5.npz')
    R, K, V = int(f['R']), int(f['K']), int(f['V'])
    ref = sgns_ref.TorchAdamRef(f['w_in0'], f['w_out0'], lr=float(f['lr']))
    torch.manual_seed(int(f['noise_seed']))
    for step in range(f['walks'].shape[0]):
        ins, tgt = sgns_ref.sg_windows(f['walks'][step].astype(np.int64), R)
        noise = generate_noise_batch(len(ins), 2 * R, K, V).numpy()
        np.testing.assert_array_equal(noise, f['noise'][step])
        loss = ref.train_step(ins, tgt, noise)
        assert loss['loss'] == pytest.approx(float(f['losses'][step][0]), rel=1e-6)
    w_in, w_out = ref.tables()
    np.testing.assert_allclose(w_in, f['w_in'], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(w_out, f['w_out'], rtol=1e-5, atol=1e-7)


def test_listscan_node2vec_equals_reference_walks():
    """The CPU baseline's node2vec (list membership at the reference's cost) replays the
    reference's R-MAT 12 walks bit-exactly, like the set-based oracle."""
    f = golden('walks_rmat12_node2vec_p0.25_q4.npz')
    g = _graph(f)
    L = int(f['walk_length'])
    for k in range(0, len(f['starts']), 8):
        w = walk_ref.node2vec_walk(g, int(f['starts'][k]), L, float(f['p']), float(f['q']),
                                   f['uniforms'][k].tolist(), listscan=True)
        np.testing.assert_array_equal(w, f['walks'][k])


@pytest.mark.parametrize('name', ['walks_karate_node2vec_p1_q0.5.npz',
                                  'walks_rmat12_node2vec_p0.25_q4.npz'])
def test_edge_class_counts_follow_the_reference_weight_rule(name):
    """oracle.walk_ref.edge_class_counts (what dw_edge_common_counts computes on the device)
    equals, for every directed edge t -> v, the number of neighbours of v the reference's rule
    (random_walk_generator.py:102-108, restated in walk_ref.node2vec_weights) weights 1/p and
    1/q at a step with prev = t — read off the weights at p = 1/2, q = 1/4 (factors 2 and 4)."""
    f = golden(name)
    g = walk_ref.CSR(f['row_ptr'], f['col'], None)   # unweighted: the factors read off as is
    cn = walk_ref.edge_class_counts(g)
    n = len(g.row_ptr) - 1
    for t in range(n):
        for e in range(g.row_ptr[t], g.row_ptr[t + 1]):
            _, w = walk_ref.node2vec_weights(g, t, g.col[e], 0.5, 0.25)
            assert int(cn[e]) >> 31 == sum(1 for x in w if x == 2.0)
            assert int(cn[e]) & 0x7FFFFFFF == sum(1 for x in w if x == 4.0)
    assert (cn >> 31 == 1).all()          # undirected: t is always a neighbour of v


@pytest.mark.parametrize('name', ['walks_karate_node2vec_p1_q0.5.npz',
                                  'walks_rmat12_node2vec_p0.25_q4.npz'])
def test_edge_class_positions_fast_equals_direct(name):
    """The hub-graph restatement (list intersection) equals the direct scan on undirected
    graphs."""
    f = golden(name)
    g = walk_ref.CSR(f['row_ptr'], f['col'], None)
    for a, b in zip(walk_ref.edge_class_positions(g), walk_ref.edge_class_positions_fast(g)):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('name', ['walks_karate_node2vec_p1_q0.5.npz',
                                  'walks_rmat12_node2vec_p0.25_q4.npz'])
def test_edge_class_positions_follow_the_reference_weight_rule(name):
    """oracle.walk_ref.edge_class_positions (what dw_n2v_edge_index_build stores: t's position
    in N(v) and the ascending positions of the 1/q neighbours) reads, for every directed edge
    t -> v, exactly the positions the reference's rule weights 1/p and 1/q (factors 2 and 4 at
    p = 1/2, q = 1/4), and agrees with the class counts."""
    f = golden(name)
    g = walk_ref.CSR(f['row_ptr'], f['col'], None)
    off, pos, pos_t = walk_ref.edge_class_positions(g)
    cn = walk_ref.edge_class_counts(g)
    n = len(g.row_ptr) - 1
    for t in range(n):
        for e in range(g.row_ptr[t], g.row_ptr[t + 1]):
            _, w = walk_ref.node2vec_weights(g, t, g.col[e], 0.5, 0.25)
            q_pos = [i for i, x in enumerate(w) if x == 4.0]
            p_pos = [i for i, x in enumerate(w) if x == 2.0]
            assert pos[off[e]:off[e + 1]].tolist() == q_pos
            assert (pos_t[e] == p_pos[0]) if p_pos else pos_t[e] == -1
            assert off[e + 1] - off[e] == int(cn[e]) & 0x7FFFFFFF
