"""The deterministic accumulation mode (word2vec/exact.py; SURVEY.md §5 "race detection").

Every gradient term enters an int64 accumulator as a fixed-point integer, so the gradients — and
the tables Adam makes of them — are the same bits whatever the order of the atomics, the
chunking of the records, a graph replay or the number of ranks:
  * the exact gradients sit within the float64 closed form's bars (the oracle);
  * the same step twice gives bit-identical gradients and tables (the float mode does not);
  * owner parts (any number of owners, centre sums kept as integers) add up to the single
    launch bit for bit;
  * two ranks (gloo on one GPU) training with OwnerTables equal one process bit for bit;
  * tools/train.py's C2-shape loop: two eager runs and the graph-replayed run end with
    bit-identical tables.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sgns_ref
from shallow_encoders import _native
from shallow_encoders.word2vec import exact
from shallow_encoders.word2vec.sgns import sgns_accumulate, sgns_owner_pass1, sgns_owner_pass2

pytestmark = pytest.mark.gpu


def _batch(V, d, n, L, R, K, seed):
    rng = np.random.default_rng(seed)
    w_in0, w_out0 = sgns_ref.xavier_tables(V, d, seed=seed)
    walks = rng.integers(0, V, size=(n, L)).astype(np.int32)
    walks[:, ::3] = 7                      # a hub row straddling many gather chunks
    ins, tgt = sgns_ref.sg_windows(walks, R)
    noise = rng.integers(0, V, size=(len(ins), 2 * R, K))
    return w_in0, w_out0, walks, ins, tgt, noise


def _exact_grads(w_in, w_out, wk, nz, R, K, scale):
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    reg = exact.Registry()
    reg.ensure(0, g_in, scale)
    reg.ensure(1, g_out, scale)
    acc = sgns_accumulate(w_in, w_out, g_in, g_out, K, walks=wk, context_radius=R, noise=nz)
    torch.cuda.synchronize()
    reg.release()
    return g_in, g_out, acc


@pytest.mark.parametrize('d', [64, 128, 40])
def test_exact_gradients_vs_oracle_and_repeatable(d, hip_device):
    """The exact gradients (g16 pass 1 for d % 64 == 0, the 64-lane pass 1 otherwise; the
    records gather) are within the float64 closed form's bars, and bit-identical run to run."""
    V, R, K, L, n = 3001, 3, 4, 30, 96
    w_in0, w_out0, walks, ins, tgt, noise = _batch(V, d, n, L, R, K, d)
    w_in, w_out = torch.as_tensor(w_in0).cuda(), torch.as_tensor(w_out0).cuda()
    wk, nz = torch.as_tensor(walks).cuda(), torch.as_tensor(noise).cuda()
    scale = 1.0 / (len(ins) * 2 * R)
    g_in, g_out, acc = _exact_grads(w_in, w_out, wk, nz, R, K, scale)
    loss, gi_ref, go_ref = sgns_ref.sgns_grads_closed_form(w_in0, w_out0, ins, tgt, noise)
    gmax = float(np.abs(gi_ref).max())
    np.testing.assert_allclose(g_in.cpu().numpy(), gi_ref, rtol=1e-4, atol=1e-6 * gmax)
    np.testing.assert_allclose(g_out.cpu().numpy(), go_ref, rtol=1e-4, atol=1e-6 * gmax)
    for _ in range(2):
        g_in2, g_out2, _ = _exact_grads(w_in, w_out, wk, nz, R, K, scale)
        assert torch.equal(g_in, g_in2) and torch.equal(g_out, g_out2)


@pytest.mark.parametrize('W', [2, 3, 8])
def test_exact_owner_parts_equal_single_launch(W, hip_device):
    """W owners' pass 1 into one int64 centre accumulator (DW_EXACT_DEFER, converted once) and
    their pass 2 slices equal the single launch's exact gradients bit for bit: the sums do not
    depend on how the terms are split."""
    V, d, R, K, L, n = 2003, 128, 2, 5, 24, 64
    w_in0, w_out0, walks, ins, tgt, noise = _batch(V, d, n, L, R, K, 5)
    w_in, w_out = torch.as_tensor(w_in0).cuda(), torch.as_tensor(w_out0).cuda()
    wk, nz = torch.as_tensor(walks).cuda(), torch.as_tensor(noise).cuda()
    scale = 1.0 / (len(ins) * 2 * R)
    g_in, g_out, _ = _exact_grads(w_in, w_out, wk, nz, R, K, scale)
    S = -(-V // W)
    g_in_parts = torch.zeros_like(w_in)
    reg = exact.Registry()
    fx_in = reg.ensure(0, g_in_parts, scale, defer=True)
    for r in range(W):
        rows = torch.arange(S, device='cuda') * W + r
        keep = rows < V
        w_loc = torch.zeros((S, d), dtype=torch.float32, device='cuda')
        w_loc[keep] = w_out[rows[keep]]
        g_loc = torch.zeros_like(w_loc)
        reg.ensure(1, g_loc, scale)
        sgns_owner_pass1(w_in, w_loc, g_in_parts, K, walks=wk, context_radius=R, owner=r,
                         n_owners=W, vocab_size=V, noise=nz, grad_scale=scale)
        sgns_owner_pass2(w_in, w_loc, g_loc, K, walks=wk, context_radius=R)
        torch.cuda.synchronize()
        assert torch.equal(g_loc[keep], g_out[rows[keep]])
    assert float(g_in_parts.abs().max()) == 0.0        # deferred: still in the integers
    fx_in.convert()
    torch.cuda.synchronize()
    reg.release()
    assert torch.equal(g_in_parts, g_in)


def test_exact_tables_repeatable(hip_device):
    """ShardedTables' fused one-GPU step (pass 1, the in-table Adam on the side stream, the
    output phase with its Adam fused) over 6 steps: bit-identical tables and Adam state from
    two runs in the deterministic mode."""
    from shallow_encoders.word2vec.sharding import ShardedTables, replicated_step
    V, d, R, K, L, n, steps = 4000, 128, 3, 5, 40, 256, 6
    g = torch.Generator().manual_seed(3)
    walks = torch.randint(1, V, (steps, n, L), generator=g, dtype=torch.int32)
    walks[:, :, ::5] = 9
    per = L - 2 * R
    scale = 1.0 / (n * per * 2 * R)

    def run(det):
        t = ShardedTables(V, d, hip_device, lr=0.01, init_seed=2)
        if det:
            t.enable_exact(scale)
        acc = torch.zeros(4, dtype=torch.float64, device=hip_device)
        st = torch.zeros(1, dtype=torch.int32, device=hip_device)
        for s in range(steps):
            replicated_step(t, walks[s].cuda(), R, K, seed=5, noise_offset=s * n * per,
                            grad_scale=scale, loss_acc=acc, status=st)
        torch.cuda.synchronize()
        _native.check_status(st, 'replicated_step')
        return [x.cpu().clone() for x in (t.w_in, t.w_out, t.m[0, :V], t.v[0, :V], t.m[1, :V],
                                          t.v[1, :V])]

    a, b = run(True), run(True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.parametrize('form', ['sequential', 'pipelined'])
def test_exact_lazy_rows_major_repeatable_and_equal_dense(form, hip_device):
    """OwnerLazyTables on one rank with the lazy Adam of both tables (the rows-major out step,
    the reference's small-batch path) in the deterministic mode: two runs give bit-identical
    tables and Adam state, and they equal the dense deterministic step's (ShardedTables:
    every row's Adam every step) bit for bit once flushed — the integer sums make the claim's
    record order irrelevant, and the lazy replays are the dense g = 0 steps. 'pipelined':
    owner_lazy_steps (the next step's claims beside this one)."""
    from shallow_encoders.word2vec.sharding import (OwnerLazyTables, ShardedTables,
                                                    owner_lazy_step, owner_lazy_steps,
                                                    replicated_step)
    # (V: a step's 65K slots leave about half the out rows untouched, so out rows fall behind
    # and k_out_rows replays their deferred steps; at V = 4,000 every row was touched every step)
    V, d, R, K, L, n, steps = 100_000, 128, 3, 5, 40, 64, 6
    g = torch.Generator().manual_seed(3)
    walks = torch.randint(1, V, (steps, n, L), generator=g, dtype=torch.int32)
    walks[:, :, ::5] = 9                     # a hub out row straddling the out-rows chunks
    per = L - 2 * R
    scale = 1.0 / (n * per * 2 * R)
    offs = [s * n * per for s in range(steps)]

    def lazy():
        t = OwnerLazyTables(V, d, hip_device, lr=0.01, init_seed=2, emulate_world=1,
                            lazy_out=True)
        t.enable_exact(scale)
        assert t.rows_major_ok(R, K) and t.pipeline_ok(R, K)
        acc = torch.zeros(4, dtype=torch.float64, device=hip_device)
        st = torch.zeros(1, dtype=torch.int32, device=hip_device)
        owner_lazy_step(t, walks[0].cuda(), R, K, seed=5, noise_offset=0, grad_scale=scale,
                        loss_acc=acc, status=st)
        if form == 'pipelined':
            owner_lazy_steps(t, [walks[s].cuda() for s in range(1, steps)], R, K, seed=5,
                             noise_offsets=offs[1:], grad_scale=scale, loss_acc=acc,
                             status=st)
        else:
            for s in range(1, steps):
                owner_lazy_step(t, walks[s].cuda(), R, K, seed=5, noise_offset=offs[s],
                                grad_scale=scale, loss_acc=acc, status=st)
        torch.cuda.synchronize()
        _native.check_status(st, 'owner_lazy_step')
        t.flush()
        return [x.cpu().clone() for x in (t.params_in[0, :V], t.w_out[:V], t.m_in[:V],
                                          t.v_in[:V], t.m_out[:V], t.v_out[:V])]

    def dense():
        t = ShardedTables(V, d, hip_device, lr=0.01, init_seed=2)
        t.enable_exact(scale)
        acc = torch.zeros(4, dtype=torch.float64, device=hip_device)
        st = torch.zeros(1, dtype=torch.int32, device=hip_device)
        for s in range(steps):
            replicated_step(t, walks[s].cuda(), R, K, seed=5, noise_offset=offs[s],
                            grad_scale=scale, loss_acc=acc, status=st)
        torch.cuda.synchronize()
        _native.check_status(st, 'replicated_step')
        return [x.cpu().clone() for x in (t.w_in, t.w_out, t.m[0, :V], t.v[0, :V], t.m[1, :V],
                                          t.v[1, :V])]

    a, b, c = lazy(), lazy(), dense()
    names = ('w_in', 'w_out', 'm_in', 'v_in', 'm_out', 'v_out')
    for name, x, y in zip(names, a, b):
        assert torch.equal(x, y), f'{name}: two lazy runs differ'
    for name, x, y in zip(names, a, c):
        diff = int((x != y).sum())
        assert diff == 0, f'{name}: {diff} entries differ from the dense deterministic step'


@pytest.mark.parametrize('path', ['dense', 'lazy'])
@pytest.mark.parametrize('table', ['in', 'out'])
@pytest.mark.parametrize('value', ['nan', 'huge'])
def test_exact_range_flags_nan_and_huge_terms(path, table, value, hip_device):
    """A gradient term past the fixed-point range — a NaN from a diverged row, or a finite term
    with |t| 2^frac >= 2^51 — sets DW_S_FIXED_RANGE and the step's status check raises
    OverflowError, in every EXACT kernel: 'dense' (ShardedTables: k_sgns_g16's centre sums over
    out rows, k_rec_gather's out sums over centre rows), 'lazy' (the rows-major step: k_out_rows
    over centre rows, the COEFIN centre pass over out rows). Element 0 of the other table is
    zeroed, so the logits stay finite and moderate and only the terms carry the bad value (a NaN
    would otherwise also poison the coefficient, a huge logit saturate it to 0)."""
    from shallow_encoders.word2vec.sharding import (OwnerLazyTables, ShardedTables,
                                                    owner_lazy_step, replicated_step)
    V, d, R, K, L, n = 600, 128, 2, 2, 20, 16
    g = torch.Generator().manual_seed(11)
    walks = torch.randint(1, V, (n, L), generator=g, dtype=torch.int32)
    node = int(walks[0, 5])
    per = L - 2 * R
    scale = 1.0 / (n * per * 2 * R)
    w_in, w_out = sgns_ref.xavier_tables(V, d, seed=4)
    w_in, w_out = torch.as_tensor(w_in).clone(), torch.as_tensor(w_out).clone()
    bad = float('nan') if value == 'nan' else 2.0 ** 24   # 2^24 * coef * 2^frac >> 2^51
    if table == 'in':
        w_in[node, 0], w_out[:, 0] = bad, 0.0
    else:
        w_out[node, 0], w_in[:, 0] = bad, 0.0
    acc = torch.zeros(4, dtype=torch.float64, device=hip_device)
    st = torch.zeros(1, dtype=torch.int32, device=hip_device)
    wk = walks.cuda()
    if path == 'dense':
        t = ShardedTables(V, d, hip_device, lr=0.01, init_seed=2)
        t.load_(w_in.cuda(), w_out.cuda())
        t.enable_exact(scale)
        replicated_step(t, wk, R, K, seed=5, noise_offset=0, grad_scale=scale, loss_acc=acc,
                        status=st)
    else:
        t = OwnerLazyTables(V, d, hip_device, lr=0.01, init_seed=2, emulate_world=1,
                            lazy_out=True)
        t.load_(w_in.cuda(), w_out.cuda())
        t.enable_exact(scale)
        assert t.rows_major_ok(R, K)
        owner_lazy_step(t, wk, R, K, seed=5, noise_offset=0, grad_scale=scale, loss_acc=acc,
                        status=st)
    torch.cuda.synchronize()
    with pytest.raises(OverflowError):
        _native.check_status(st, f'{path} step')


# ---- two ranks on one GPU (gloo), deterministic mode: bit-identical to one process ---------
V2, D2, R2, K2, L2, NW2, STEPS2, LR2 = 900, 64, 2, 3, 14, 48, 4, 5e-3


def _walks2():
    g = torch.Generator().manual_seed(21)
    w = torch.randint(1, V2, (STEPS2, NW2, L2), generator=g, dtype=torch.int32)
    w[:, :, ::4] = 3
    return w


def _scale2():
    return 1.0 / (NW2 * (L2 - 2 * R2) * 2 * R2)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exact_owner_run(rank, world, port, q):
    try:
        os.environ['MASTER_ADDR'] = '127.0.0.1'
        os.environ['MASTER_PORT'] = str(port)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from shallow_encoders.word2vec.sharding import OwnerTables, owner_step
        t = OwnerTables(V2, D2, 'cuda:0', lr=LR2, init_seed=4)
        t.enable_exact(_scale2())
        walks = _walks2()
        per = L2 - 2 * R2
        acc = torch.zeros(4, dtype=torch.float64, device='cuda:0')
        status = torch.zeros(1, dtype=torch.int32, device='cuda:0')
        for s in range(STEPS2):
            owner_step(t, walks[s].cuda(), R2, K2, seed=11, noise_offset=s * NW2 * per,
                       grad_scale=_scale2(), loss_acc=acc, status=status)
        torch.cuda.synchronize()
        _native.check_status(status, 'owner_step')
        full = [x.cpu().numpy().copy() for x in t.full_state()]
        q.put((rank, full, None))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report, the parent asserts
        q.put((rank, None, repr(e)))


@pytest.mark.timeout(600)
def test_exact_two_ranks_equal_single_process(hip_device):
    """OwnerTables at world 2 (gloo; the centre sums reduce-scattered as int64) and one process
    (ShardedTables) end with the same tables and Adam state, bit for bit."""
    from shallow_encoders.word2vec.sharding import ShardedTables
    ref = ShardedTables(V2, D2, hip_device, lr=LR2, init_seed=4)
    ref.enable_exact(_scale2())
    walks = _walks2()
    per = L2 - 2 * R2
    for s in range(STEPS2):
        sgns_accumulate(ref.w_in, ref.w_out, ref.g_in, ref.g_out, K2, walks=walks[s].cuda(),
                        context_radius=R2, seed=11, noise_offset=s * NW2 * per,
                        grad_scale=_scale2())
        ref.step()
    torch.cuda.synchronize()
    want = [x.cpu().numpy() for x in (ref.w_in, ref.m[0, :V2], ref.v[0, :V2], ref.w_out,
                                      ref.m[1, :V2], ref.v[1, :V2])]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_exact_owner_run, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=500) for _ in range(2)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    errs = [r[2] for r in res if r[2]]
    assert not errs, errs
    for _, full, _ in res:
        for x, y in zip(full, want):
            np.testing.assert_array_equal(x, y)


@pytest.mark.timeout(900)
def test_exact_train_loop_eager_twice_and_graphs_bit_identical(tmp_path, hip_device,
                                                              monkeypatch):
    """tools/train.py on the C2 shape (Cora-sized R-MAT, 64-walk batches, d = 128, Philox walks,
    device negatives) with DW_DETERMINISTIC=1: two eager runs and the run whose middle batches
    replay as HIP graphs (GraphedTrainerStep) end with bit-identical tables — where the float
    mode's runs end up to ~1 apart (scripts/experiments/train_graph_repro.py)."""
    from tools import train as train_tool
    monkeypatch.setenv('DW_DETERMINISTIC', '1')
    base = ['datamodule.dataset_name=graph_rmat', 'datamodule.additional_parameters.scale=12',
            'datamodule.additional_parameters.n_edges=5429',
            'datamodule.additional_parameters.graph_seed=0',
            'datamodule.additional_parameters.walks_per_node=1',
            'datamodule.additional_parameters.method_params.q=1',
            'datamodule.additional_parameters.rng=philox', 'train.noise=device',
            'model.embedding_size=128', 'train.optimizer.lr=0.01', 'train.max_epochs=2']
    states = []
    for tag, graph in (('eagerA', '0'), ('eagerB', '0'), ('graph', '1')):
        monkeypatch.setenv('DW_TRAIN_GRAPH', graph)
        monkeypatch.setenv('DW_TRAIN_GRAPH_SCATTER', 'auto')
        out = str(tmp_path / tag)
        torch.manual_seed(0)
        random.seed(0)   # the start-node shuffle (datasets.py:45,86-88: the global generator)
        train_tool.main(['--config-name', 'sge_sg_cora', f'path.output_dir={out}',
                         f'output_dir={out}', f'train.experiment={tag}'] + base)
        ck = os.path.join(out, 'graph_rmat', tag, 'checkpoints', 'last.ckpt')
        states.append(torch.load(ck, weights_only=True))
    s0 = states[0]
    assert s0['global_step'] == 128
    for s in states[1:]:
        assert s['global_step'] == s0['global_step']
        for k, v in s0['state_dict'].items():
            assert torch.equal(v, s['state_dict'][k]), k


def test_registry_keeps_accumulators_across_batch_shapes(hip_device):
    """An epoch's short last batch changes grad_scale (so frac) for one step and back: the
    registry re-registers the accumulator it already has for each (buffer, frac) instead of
    allocating and zeroing new ones, so the buffers a captured graph adds into
    stay allocated; and a step after the switch back gives the same gradients as a fresh
    registry at that shape."""
    V, d, R, K, L = 1201, 64, 2, 3, 12
    w_in0, w_out0, walks, ins, tgt, noise = _batch(V, d, 24, L, R, K, 3)
    w_in, w_out = torch.as_tensor(w_in0).cuda(), torch.as_tensor(w_out0).cuda()
    wk, nz = torch.as_tensor(walks).cuda(), torch.as_tensor(noise).cuda()
    g_in, g_out = torch.zeros_like(w_in), torch.zeros_like(w_out)
    full, short = 1.0 / tgt.size, 1.0 / (3 * tgt.size // 8)
    assert exact.frac_bits(full) != exact.frac_bits(short)
    reg = exact.Registry()
    a0 = reg.ensure(0, g_in, full)
    acc_ptr = a0.acc.data_ptr()
    b0 = reg.ensure(0, g_in, short)
    assert b0 is not a0 and not a0.active and b0.active
    a1 = reg.ensure(0, g_in, full)
    assert a1 is a0 and a1.active and not b0.active and a1.acc.data_ptr() == acc_ptr
    assert reg.live() == [a1]
    reg.ensure(1, g_out, full)
    sgns_accumulate(w_in, w_out, g_in, g_out, K, walks=wk, context_radius=R, noise=nz)
    torch.cuda.synchronize()
    reg.release()
    assert int(a1.acc.abs().sum()) == 0          # the conversion left the sums cleared
    ref_in, ref_out, _ = _exact_grads(w_in, w_out, wk, nz, R, K, full)
    assert torch.equal(g_in.view(torch.int32), ref_in.view(torch.int32))
    assert torch.equal(g_out.view(torch.int32), ref_out.view(torch.int32))
    for _ in range(2 * exact.Registry.MAX_PER_KEY):      # bounded per buffer
        reg.ensure(0, g_in, 1.0 / (tgt.size * np.random.default_rng().integers(2, 1 << 20)))
    assert len(reg._cache[0]) <= exact.Registry.MAX_PER_KEY
    reg.release()
