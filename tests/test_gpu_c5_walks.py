"""BASELINE C5's node2vec walks at their own scale: R-MAT 24 (16,777,216 nodes, 256M edge draws,
513M directed edges, hubs of 392,747 neighbours), p = .25, q = 4, over the per-edge position
index (uint16 / int32 lists, 132.6 GB, built in chunks).

  * the exact walker (dw_walk_replay_positions, the reference's pick law and arithmetic) equals
    the wave walker with the per-edge counts (DW_N2V_POS=0, the round-3 walker) bit for bit,
    from the largest hubs and from random nodes, uniforms drawn from numpy;
  * the exact walker equals the oracle's replay (oracle/walk_ref.py) bit for bit, its serial
    picks on the hub's int32 lists included;
  * the Philox walker over the index (dw_walk_fast_positions, layout='positions') equals its
    oracle (oracle/philox.fast_walks_positions) on walks through the hubs.
Skipped when the device cannot hold the index next to the graph (CSRGraph._build_n2v_index's
budget)."""
import numpy as np
import pytest
import torch

from oracle import philox as ph

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

SCALE, EDGES, P, Q = 24, 256_000_000, 0.25, 4.0


@pytest.fixture(scope='module')
def c5_index(hip_device):
    import gc
    from shallow_encoders.graph.rmat import rmat_graph
    gc.collect()
    torch.cuda.empty_cache()
    csr = rmat_graph(SCALE, EDGES, 0, device=hip_device)
    d = csr.device_tensors(hip_device, need_n2v_index=True)
    info = d.get('n2v_index_info', {})
    if d.get('n2v_rec') is None:
        pytest.skip(f'the C5 position index does not fit here: {info}')
    assert info['entries'] == 55_531_063_230 and info['chunks'] > 100, info
    yield csr
    del csr, d
    torch.cuda.empty_cache()


def _starts(csr, n_hub, n_rand, seed):
    deg = csr.degree()
    rng = np.random.default_rng(seed)
    hubs = np.argsort(-deg[1:])[:n_hub] + 1
    live = np.nonzero(deg[1:] > 0)[0] + 1
    return np.concatenate([hubs, rng.choice(live, n_rand)]).astype(np.int32)


def test_c5_exact_positions_walker_equals_wave_walker(c5_index, hip_device, monkeypatch):
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    csr = c5_index
    starts = _starts(csr, 1024, 1024, 7)
    assert csr.degree()[starts[0]] == 392_747
    L = 20
    u = torch.from_numpy(np.random.default_rng(11).random((starts.size, L - 1))).to(hip_device)
    w = Node2Vec(csr, L, p=P, q=Q, device=hip_device)
    st = torch.as_tensor(starts)
    got = w.walk_batch(st, uniforms=u).cpu().numpy()
    monkeypatch.setenv('DW_N2V_POS', '0')
    ref = w.walk_batch(st, uniforms=u).cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    assert (got >= 1).all()          # no walk aborted
    # the walks run through the hubs' int32 lists
    deg = csr.degree()
    assert (deg[got[:, 1:]] > 65_536).sum() > 100


def test_c5_exact_walker_vs_oracle(c5_index, hip_device):
    """The exact walker (dw_walk_replay_positions) against the oracle's replay
    (walk_ref.walks_replay over the host CSR, numpy-backed, the undirected membership test) at
    R-MAT 24 itself, bit for bit: walks from the 16 largest hubs (the 392,747-neighbour one
    first), from 16 random nodes, and 16 walks from neighbours t of the largest hub H whose
    first draw picks H and whose second draw lies exactly on a class boundary of the step
    t -> H — a pick the margin cannot decide, so the lane's serial arithmetic decides it over
    H's int32 position list (deg H > 65,536). A quarter of the other walks' second draws are on
    boundaries too. The counted launch shows the serial picks were taken."""
    from oracle import walk_ref
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    csr = c5_index
    rng = np.random.default_rng(29)
    L = 8
    g = walk_ref.ArrayCSR(csr.row_ptr, csr.host_col(), None, undirected=True)
    deg = csr.degree()
    hub = int(np.argmax(deg))
    assert deg[hub] == 392_747
    starts = list(_starts(csr, 16, 16, 13))
    nb_h = np.asarray(g.neighbors(hub))
    ts = rng.choice(nb_h, 16, replace=False)
    starts += [int(t) for t in ts]
    starts = np.asarray(starts, dtype=np.int32)
    u = rng.random((starts.size, L - 1))
    for w in range(32, starts.size):      # t -> H, then a boundary draw at H
        t = int(starts[w])
        nt = g.neighbors(t)
        u[w, 0] = (nt.index(hub) + 0.5) / len(nt)
        nbrs, wt = walk_ref.node2vec_weights(g, t, hub, P, Q)
        k = int(rng.integers(0, len(nbrs) - 1))
        u[w, 1] = float(np.sum(wt[:k + 1])) / float(np.sum(wt))
    for w in range(1, 32, 4):             # boundary second draws elsewhere
        s = int(starts[w])
        v1 = int(walk_ref.walks_replay(g, [s], 2, 'node2vec', P, Q, u[w:w + 1, :1])[0, 1])
        nbrs, wt = walk_ref.node2vec_weights(g, s, v1, P, Q)
        if len(nbrs) >= 2:
            k = int(rng.integers(0, len(nbrs) - 1))
            u[w, 1] = float(np.sum(wt[:k + 1])) / float(np.sum(wt))
    w = Node2Vec(csr, L, p=P, q=Q, device=hip_device)
    got = w.walk_batch(torch.as_tensor(starts), uniforms=u).cpu().numpy()
    assert w.last_walker == 'dw_walk_replay_positions'
    ref = walk_ref.walks_replay(g, starts, L, 'node2vec', P, Q, u)
    np.testing.assert_array_equal(got, ref)
    assert (got[32:, 1] == hub).all()
    c = w.count_replay_traffic(torch.as_tensor(starts), torch.from_numpy(u).to(hip_device))
    print(f'C5 exact walker vs oracle: {starts.size} walks of {L}, serial picks {c["probes"]}')
    assert c['probes'] > 0, c


def test_c5_philox_positions_walker_vs_oracle(c5_index, hip_device):
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    csr = c5_index
    starts = _starts(csr, 8, 8, 3)
    L = 6
    w = Node2Vec(csr, L, p=P, q=Q, rng='philox', seed=21, device=hip_device,
                 layout='positions')   # (C5's 132 GB index: above the 'indexed' size rule)
    got = w.walk_batch(torch.as_tensor(starts), walk_id0=1000).cpu().numpy()
    assert w.last_walker == 'dw_walk_fast_positions'
    assert not csr.philox_positions(hip_device)   # the default there: the rejection walker
    exp = ph.fast_walks_positions(csr.row_ptr, csr.host_col(), starts, L, P, Q, seed=21,
                                  walk_id0=1000)
    np.testing.assert_array_equal(got, exp)
