"""CPython's random.random() stream generated on the MI355X (dw_mt_uniforms) against CPython.

The reference's walkers consume one random.random() per step (random_walk_generator.py:68,113);
the replay walkers are fed that stream from HBM. Bar: bit-identical doubles and the identical
generator state afterwards (random.getstate()), over >= 10^8 draws, odd and even start
indices, calls that end on the state's last word, and chains that start in the middle of a
double (a double's two words in different chains).
"""
import random

import numpy as np
import pytest
import torch

from shallow_encoders import _native
from shallow_encoders.graph.rng import (draw_uniforms, draw_uniforms_device, mt_jump_table,
                                        mt_workspace)

pytestmark = pytest.mark.gpu


def _gen(seed, skip):
    r = random.Random(seed)
    for _ in range(skip):
        r.random()
    return r


def _clone(r):
    c = random.Random()
    c.setstate(r.getstate())
    return c


@pytest.mark.parametrize('seed,skip,n', [(0, 0, 1), (1, 1, 2), (2, 311, 313), (3, 312, 312),
                                         (4, 0, 624 * 300 + 7), (5, 17, 1_000_003),
                                         (6, 123, 10_000_000)])
def test_device_stream_equals_cpython(seed, skip, n, hip_device):
    r = _gen(seed, skip)
    exp_r = _clone(r)
    head = min(n, 200_000)
    exp_head = np.array([exp_r.random() for _ in range(head)])     # CPython itself
    exp = np.concatenate([exp_head, draw_uniforms(n - head, exp_r)]) if n > head else exp_head
    got = draw_uniforms_device(n, hip_device, rng=r)
    assert got.dtype == torch.float64 and got.numel() == n
    assert torch.equal(got.cpu(), torch.from_numpy(exp))
    assert r.getstate() == exp_r.getstate()
    assert r.random() == exp_r.random()


def test_device_stream_1e8_draws(hip_device):
    """>= 10^8 draws in one call (the 1M-walk C3 batch is 79M): bit-identical, state identical."""
    n = 100_000_001
    r = _gen(42, 5)
    exp_r = _clone(r)
    got = draw_uniforms_device(n, hip_device, rng=r)
    exp = torch.from_numpy(draw_uniforms(n, exp_r)).to(hip_device)
    neq = int((got != exp).sum())
    assert neq == 0, f'{neq} of {n} doubles differ'
    assert r.getstate() == exp_r.getstate()
    del exp, got


@pytest.mark.parametrize('stride,seed,skip,n', [(1, 7, 0, 5000), (1, 8, 1, 5000),
                                                (2, 9, 311, 3001), (3, 10, 623, 2000),
                                                (1, 11, 3, 312 * 5)])
def test_multi_chain_boundaries(stride, seed, skip, n, hip_device):
    """Small window strides force many chains (each seeded by a jump) on short streams: doubles
    straddling windows and chains at odd indices, the final state from the last chain."""
    r = _gen(seed, skip)
    exp_r = _clone(r)
    exp = np.array([exp_r.random() for _ in range(n)])
    internal = np.asarray(r.getstate()[1], dtype=np.uint32)
    index = int(internal[624])
    windows = (index + 2 * n - 1) // 624 + 1
    chains = -(-windows // stride)
    assert chains > 1
    pos, off, n_tab = mt_jump_table(hip_device, stride, chains)
    mt = torch.from_numpy(internal[:624].view(np.int32).copy()).to(hip_device)
    out = torch.full((n,), float('nan'), dtype=torch.float64, device=hip_device)
    st = torch.zeros(625, dtype=torch.int32, device=hip_device)
    ws = mt_workspace(hip_device, chains)
    _native.call('dw_mt_uniforms', _native.ptr(mt), index, n, _native.ptr(out), _native.ptr(st),
                 stride, _native.ptr(pos), _native.ptr(off), n_tab, _native.ptr(ws), ws.numel(),
                 _native.stream(hip_device))
    np.testing.assert_array_equal(out.cpu().numpy(), exp)
    new = st.cpu().numpy().view(np.uint32)
    ref = exp_r.getstate()[1]
    assert tuple(int(v) for v in new) == ref


def test_abi_rejects_short_jump_table(hip_device):
    mt = torch.zeros(624, dtype=torch.int32, device=hip_device)
    out = torch.empty(10_000, dtype=torch.float64, device=hip_device)
    st = torch.empty(625, dtype=torch.int32, device=hip_device)
    with pytest.raises(_native.DWError):
        _native.call('dw_mt_uniforms', _native.ptr(mt), 0, 10_000, _native.ptr(out),
                     _native.ptr(st), 1, None, None, 0, None, 0, _native.stream(hip_device))
    with pytest.raises(_native.DWError):
        _native.call('dw_mt_uniforms', _native.ptr(mt), 625, 1, _native.ptr(out),
                     _native.ptr(st), 256, None, None, 0, None, 0, _native.stream(hip_device))


@pytest.mark.parametrize('method', ['deepwalk', 'node2vec'])
def test_walker_default_stream_is_device_generated_and_exact(method, hip_device):
    """walk_batch without uniforms draws the global stream on the device: the same walks as the
    host-drawn uniforms, and the global generator left where the reference would leave it."""
    from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec
    from shallow_encoders.graph.rmat import rmat_graph
    csr = rmat_graph(14, 150_000, 0, device=hip_device)
    L = 20
    w = (Node2Vec(csr, L, p=0.25, q=4, device=hip_device) if method == 'node2vec'
         else DeepWalk(csr, L, device=hip_device))
    starts = torch.arange(1, 5001, dtype=torch.int32)
    random.seed(77)
    got = w.walk_batch(starts).cpu().numpy()
    after = random.getstate()
    random.seed(77)
    u = draw_uniforms(5000 * (L - 1))
    exp = w.walk_batch(starts, uniforms=u).cpu().numpy()
    np.testing.assert_array_equal(got, exp)
    assert random.getstate() == after


# ---- a generator held in HBM (DeviceMT / dw_mt_draw): torch's negatives and CPython's walks ---
def _torch_expected(seed, skip, high, sizes):
    """torch.randint draws of the given sizes after torch.manual_seed(seed) and `skip` draws, and
    torch's generator state after them (CPU; the reference's generate_noise_batch)."""
    torch.manual_seed(seed)
    if skip:
        torch.randint(0, 7, (skip,))
    st0 = torch.get_rng_state()
    exp = [torch.randint(0, high, (n,), dtype=torch.long) for n in sizes]
    return st0, exp, torch.get_rng_state()


@pytest.mark.parametrize('seed,skip,high,sizes', [
    (0, 0, 1_048_577, [4480 * 50] * 6),            # the reference's 64-walk C3 batches
    (1, 311, 2708, [1, 623, 624, 625, 9_999]),      # Cora-sized vocabulary, window edges
    (2, 5, 2 ** 28 + 11, [3, 1000, 77_777]),        # two outputs per value
    (3, 0, 1_048_577, [10_000_001]),                # >= 10^7 draws in one call
])
def test_device_torch_randint_equals_torch(seed, skip, high, sizes, hip_device):
    """DeviceMT.randint (dw_mt_draw mode 1 / 2) from torch's CPU generator state
    gives torch.randint's values bit for bit, call after call, with the state kept in HBM between
    calls; to_torch() leaves torch.get_rng_state() equal to what the host draws leave."""
    from shallow_encoders.graph.rng import DeviceMT
    st0, exp, st1 = _torch_expected(seed, skip, high, sizes)
    torch.set_rng_state(st0)
    g = DeviceMT.from_torch(hip_device)
    for n, e in zip(sizes, exp):
        got = g.randint(high, n)
        assert torch.equal(got.cpu(), e), n
    g.to_torch()
    assert torch.equal(torch.get_rng_state(), st1)


def test_device_torch_randint_device_index_and_graph(hip_device):
    """The index read on the device (device_index=True) and the draws captured once in a HIP
    graph and replayed: the same stream as torch.randint, replay after replay (the graphed
    training loop's negatives)."""
    from shallow_encoders.graph.rng import DeviceMT
    high, n, reps = 1_048_577, 4480 * 50, 5
    st0, exp, st1 = _torch_expected(4, 3, high, [n] * (reps + 1))
    torch.set_rng_state(st0)
    g = DeviceMT.from_torch(hip_device, device_index=True)
    out = torch.empty(n, dtype=torch.int64, device=hip_device)
    g.randint(high, n, out=out)                       # eager, device index
    assert torch.equal(out.cpu(), exp[0])
    s = torch.cuda.Stream(hip_device)
    s.wait_stream(torch.cuda.current_stream(hip_device))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        g.randint(high, n, out=out)
    for k in range(reps):
        graph.replay()
        torch.cuda.synchronize(hip_device)
        assert torch.equal(out.cpu(), exp[k + 1]), k
    g.to_torch()
    assert torch.equal(torch.get_rng_state(), st1)


@pytest.mark.parametrize('device_index', [False, True])
def test_device_mt_uniforms_resident_equals_cpython(device_index, hip_device):
    """DeviceMT.uniforms: CPython's random.random() stream call after call with the state in
    HBM (no host round trip; the host follows the index, or the device reads it), then handed
    back to `random` exactly."""
    from shallow_encoders.graph.rng import DeviceMT
    r = _gen(31, 7)
    exp_r = _clone(r)
    g = DeviceMT.from_random(hip_device, rng=r, device_index=device_index)
    for n in (1, 311, 312, 647_168, 5):
        got = g.uniforms(n)
        exp = draw_uniforms(n, exp_r) if n >= 64 else np.array([exp_r.random() for _ in range(n)])
        assert torch.equal(got.cpu(), torch.from_numpy(exp)), n
    g.to_random(r)
    assert r.getstate() == exp_r.getstate()
