"""Benchmark: DeepWalk/node2vec SGNS training on the synthetic 1M-node R-MAT graph (BASELINE C3/C4).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-walks B] ...
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (N > 1)

One step = one pass of the hot path over one batch of synthetic input, all on the device:
  1. B walks of length 80 from the Philox fast walker (start node = global walk id // 10, i.e.
     node-id order x 10 walks per node, over successive steps);
  2. the fused SGNS kernel (R=5 windows, K=5 uniform device negatives, d=128) accumulating the
     dense gradient of the batch-mean loss into both tables;
  3. dense Adam over both full 1,048,577 x 128 tables (torch.optim.Adam semantics), with the
     node-id-range sharded reduce-scatter / all-gather exchange over RCCL when N > 1.
Weak scaling (default): every rank processes B walks per step; `--scaling strong`: the global
batch is B walks and every rank trains 1/N of it. `value` = positive pairs of ALL ranks / s.

Also reported: walks/s of the walker alone (DeepWalk and node2vec p=.25 q=4), the SGNS kernel
against the HBM roofline (algorithmic bytes / live HIP-event kernel time), and the CPU
baseline (the oracle = reference-algorithm restatement, rank 0 at N=1, bounded sample).
"""
import argparse
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'deepwalk-and-node2vec_amd'))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


CONFIGS = {
    # BASELINE C2 shape (Cora is not shipped): a 4,096-node R-MAT with Cora's 5,429 edges, the
    # reference's Cora config (node2vec, L=10, R=2, 16 walks per node, 64-walk batches) at d=128
    'c2': dict(scale=12, edges=5429, dim=128, method='node2vec', p=1.0, q=1.0, radius=2,
               walk_length=10, batch_walks=64, walks_per_node=16),
    'c3': dict(scale=20, edges=10_000_000, dim=128, method='deepwalk', p=1.0, q=1.0, radius=5,
               walk_length=80, batch_walks=8192, walks_per_node=10),
    'c5': dict(scale=24, edges=256_000_000, dim=256, method='node2vec', p=0.25, q=4.0, radius=5,
               walk_length=80, batch_walks=8192, walks_per_node=10),
}


def measured_copy_gbs(dev, nbytes: int = 2 << 30, reps: int = 5) -> float:
    """STREAM copy on this GPU (dw_stream_copy, float4 lanes): bytes read + written per second,
    best of `reps` — the measured HBM roofline reported beside the 8 TB/s spec figure."""
    from shallow_encoders import _native
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).uniform_()
    dst = torch.empty_like(src)
    best = None
    with torch.cuda.device(dev):
        for _ in range(reps + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _native.call('dw_stream_copy', _native.ptr(src), _native.ptr(dst), nbytes,
                         _native.stream(dev))
            e1.record()
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
    del src, dst
    torch.cuda.empty_cache()
    return 2 * nbytes / (best * 1e-3) / 1e9


def sgns_bytes_per_pair(d: int, K: int, R: int) -> float:
    """Algorithmic HBM bytes per positive pair: every gathered fp32 row read
    once and its gradient written once; int64 ids. 6,295 B at d=128, K=5, R=5."""
    return 8 * d * (1 + K) + 8 * d / (2 * R) + 8 * (1 + K) + 8 / (2 * R)


def walk_line_rates(table_bytes: int):
    """The random-line rates measured on MI355X by scripts/microbench/random_lines.hip
    (profiles/r02_random_lines.json) for the table size nearest ``table_bytes``: independent
    16-B gathers and 1M dependent chains over a table of 16-B entries."""
    path = os.path.join(REPO, 'profiles', 'r02_random_lines.json')
    try:
        with open(path) as f:
            rows = [json.loads(x) for x in f if x.strip().startswith('{')]
    except OSError:
        return None
    if not rows:
        return None
    mib = table_bytes / 2 ** 20
    r = min(rows, key=lambda x: abs(math.log(x['table_MiB'] / mib)))
    return dict(r, source=f'profiles/r02_random_lines.json ({r["table_MiB"]} MiB table)')


def dependent_line_roofline(steps: int, kern_s: float, lines_per_step: float, table_bytes: int,
                            what: str):
    """A latency-bound walker's random-line bound: ``lines_per_step`` dependent line loads per
    step (from the walker's counted launch of the same walks) x steps / kernel time, against
    the dependent-chain rate measured for a table of that size (walk_line_rates). frac_of_chase
    near 1: the walker runs at the chip's rate of dependent random lines, not bound by bytes."""
    rate = walk_line_rates(table_bytes)
    if not rate:
        return None
    lines_s = steps * lines_per_step / kern_s
    return {'steps_per_s': steps / kern_s, 'dependent_lines_per_step': lines_per_step,
            'dependent_lines_per_s': lines_s,
            'chase_lines_per_s': rate['chase_lines_per_s'],
            'gather_lines_per_s': rate['gather_lines_per_s'],
            'frac_of_chase': lines_s / rate['chase_lines_per_s'],
            'lines': what, 'source': rate['source']}


_RESULT = {}   # run()'s JSON line, printed by main()
# the position walkers' dependent lines per step: the edge's 32-B record, then each move of the
# pick's binary search to another 128-B line of the position list (counted launch)
POS_LINES = 'edge record + the position search\'s line moves'



def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def cpu_baseline(csr, args, budget_s: float, walk_methods):
    """The oracle port of the reference's CPU path (cross-checked against the reference itself
    in the build container: identical outputs; speed in profiles/r02_cpu_crosscheck.log), timed
    on this host on bounded samples of the same workload:
      * SGNS steps (torch-CPU restatement of model.py / loss.py + autograd + torch.optim.Adam,
        the whole V x d tables) at the reference configs' 64 walks per step and at the GPU
        line's batch (like-for-like: ``value``);
      * the walkers, 1 core, with the reference's per-step work on networkx's adjacency layout
        (oracle NxLikeGraph): DeepWalk and node2vec with the GPU walk bench's (p, q)."""
    from oracle import sgns_ref, walk_ref
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    V, d, R, K, L = csr.vocab_size, args.dim, args.radius, args.neg, args.walk_length
    rng = np.random.default_rng(0)
    w_in, w_out = sgns_ref.xavier_tables(V, d, seed=0)
    ref = sgns_ref.TorchAdamRef(w_in, w_out, lr=args.lr)

    def batch(bw):
        walks = torch.from_numpy(rng.integers(1, V, size=(bw, L)).astype(np.int32))
        ins, tgt = sgns_ref.sg_windows_torch(walks, R)
        return ins.numpy(), tgt.numpy(), rng.integers(0, V, size=(ins.shape[0], 2 * R, K))

    ref.train_step(*batch(64))                 # allocates the Adam state
    samples = []
    for bw in sorted({64, args.batch_walks}):
        ins, tgt, noise = batch(bw)
        steps, t = 0, 0.0
        while steps < 1 or (bw == 64 and t < 0.3 * budget_s):
            a = time.perf_counter()
            ref.train_step(ins, tgt, noise)
            t += time.perf_counter() - a
            steps += 1
            if bw == 64:
                ins, tgt, noise = batch(bw)
        samples.append({'batch_walks': bw, 'pairs_per_step': int(tgt.size), 'steps': steps,
                        'seconds': t, 'pairs_per_s': steps * tgt.size / t})
    del ref
    a = time.perf_counter()
    g = walk_ref.NxLikeGraph(csr.row_ptr, csr.host_col(), csr.itos)
    build_s = time.perf_counter() - a
    names = csr.itos
    walkers = {}
    for meth, p, q in walk_methods:
        # node2vec at C3 costs seconds per walk (a hub step scans ~44K neighbour lists): time
        # steps of length-10 walks from uniform starts and quote walks of L as steps / (L-1)
        wl = L if meth == 'deepwalk' else min(L, 10)
        steps, a = 0, time.perf_counter()
        while steps == 0 or time.perf_counter() - a < 0.2 * budget_s:
            s0 = names[int(rng.integers(1, V))]
            u = rng.random(wl - 1).tolist()
            if meth == 'deepwalk':
                walk_ref.deepwalk_walk(g, s0, wl, u)
            else:
                walk_ref.node2vec_walk(g, s0, wl, p, q, u, listscan=True)
            steps += wl - 1
        dt = time.perf_counter() - a
        walkers[meth] = {'p': p, 'q': q, 'sample_walk_length': wl, 'steps': steps,
                         'seconds': dt, 'steps_per_s': steps / dt,
                         'walks_per_s': steps / dt / (L - 1)}
    del g
    like = next(x for x in samples if x['batch_walks'] == args.batch_walks)
    return {
        'value': like['pairs_per_s'], 'unit': 'positive-pairs/s', 'cores': threads, 'kind': 'port',
        'sample': (f'oracle SGNS step (torch-CPU restatement of model.py/loss.py + autograd + '
                   f'torch.optim.Adam over the whole V={V} x d={d} tables, K={K}, R={R}, L={L}) at '
                   f'the GPU line\'s {args.batch_walks} walks/step ({like["steps"]} step(s), '
                   f'{like["seconds"]:.1f}s) and at the reference configs\' 64 walks/step, '
                   f'{threads} torch threads; walkers: the reference\'s per-step algorithm on '
                   f'networkx\'s adjacency layout (built in {build_s:.1f}s), 1 core, '
                   f'{0.2 * budget_s:.0f}s each'),
        'batches': samples,
        'walkers': walkers,
        'walks_per_s': {m: w['walks_per_s'] for m, w in walkers.items()},
    }


def batch64_line(csr, args, dev, epoch_starts, copy_gbs: float, n_steps: int) -> dict:
    """The reference configs' own batch (configs/sge_sg_cora.yaml:24, sge_sg_karate_club.yaml:24:
    64 walks per step) on the headline graph, timed by the driver's run.

    The one-GPU composition bench.py takes for that shape (`--batch-walks 64`): OwnerLazyTables
    on one rank with the lazy exact Adam of both tables (only the rows a step touches are read
    and updated; deferred g = 0 steps replayed bit-exactly), the records placed by the claim and
    the rows-major out step, replayed as HIP graphs of 16 pipelined steps (GraphedOwnerStep /
    owner_lazy_steps: the next step's placement and in-row catch-up beside this one) with the
    Philox walker in front; `--deterministic` runs it with the integer sums. After the timed replays one more step is run eagerly from a
    flushed pre-state and checked on ~256 in and ~256 out rows against the float64 restatement
    (word2vec/verify.py; the parity tests' single-step bars); a miss fails the bench.

    roofline: SURVEY §8d's per-pair SGNS bytes plus the dense-Adam figure (7 x 4 B per entry)
    on the rows the step touches (the checked step's |U| in rows and stepped out rows), over the
    HIP-event window of the replays."""
    from shallow_encoders import _native
    from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec
    from shallow_encoders.word2vec import verify
    from shallow_encoders.word2vec.graphed import GraphedOwnerStep
    from shallow_encoders.word2vec.sgns import loss_terms
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    V, d, R, K, L = csr.vocab_size, args.dim, args.radius, args.neg, args.walk_length
    B, unroll, warm, seed = 64, 16, 8, 99
    n_steps = max(unroll, n_steps // unroll * unroll)
    per = L - 2 * R
    pairs = B * per * 2 * R
    grad_scale = 1.0 / pairs
    walks_total = (V - 1) * args.walks_per_node
    walker = (Node2Vec(csr, L, p=args.p, q=args.q, rng='philox', seed=1234, device=dev)
              if args.method == 'node2vec' else DeepWalk(csr, L, rng='philox', seed=1234,
                                                         device=dev))
    tables = OwnerLazyTables(V, d, dev, lr=args.lr, init_seed=0, lazy_out=True)
    if args.deterministic:   # the integer sums of the rows-major step (word2vec/exact.py)
        tables.enable_exact(grad_scale)
    loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)

    def eager_step(s: int) -> torch.Tensor:
        g0 = s * B
        a = g0 % walks_total
        walks = walker.walk_batch(epoch_starts[a:a + B], walk_id0=g0, check=False,
                                  status=status)
        owner_lazy_step(tables, walks, R, K, seed=seed, noise_offset=g0 * per,
                        grad_scale=grad_scale, loss_acc=loss_acc, status=status)
        return walks

    for s in range(warm):
        eager_step(s)
    long_steps = max(int(getattr(args, 'batch64_long', 0) or 0), 0) // unroll * unroll
    total = max(n_steps, long_steps)
    graphed = GraphedOwnerStep(tables, walker, epoch_starts, B, R, K, seed=seed,
                               grad_scale=grad_scale, loss_acc=loss_acc, status=status,
                               first_walk_id=warm * B, n_steps=total + unroll, unroll=unroll)
    graphed.replay()                      # one untimed replay (first-launch costs)
    torch.cuda.synchronize(dev)
    loss_acc.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a = time.perf_counter()
    e0.record()
    for _ in range(n_steps // unroll):
        graphed.replay()
    e1.record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - a
    _native.check_status(status, 'bench batch64')
    kern_ms = e0.elapsed_time(e1) / n_steps
    mean_loss = float(loss_terms(loss_acc, pairs * n_steps, K)['loss'])

    # the steady state: the same replays on to `long_steps`, the last 4,000 timed (the step
    # check below then runs from that state)
    steady = None
    if long_steps > n_steps:
        rest = long_steps - n_steps
        win = min(rest, 4000 // unroll * unroll)
        for _ in range((rest - win) // unroll):
            graphed.replay()
        torch.cuda.synchronize(dev)
        a2 = time.perf_counter()
        for _ in range(win // unroll):
            graphed.replay()
        torch.cuda.synchronize(dev)
        el2 = time.perf_counter() - a2
        _native.check_status(status, 'bench batch64 steady state')
        steady = {'steps_before': warm + unroll + n_steps + rest - win, 'steps': win,
                  'ms_per_step': el2 / win * 1e3, 'value': pairs * win / el2,
                  'unit': 'positive-pairs/s'}
        n_done = n_steps + rest
    else:
        n_done = n_steps

    # one more step, eager, checked from its (flushed) pre-state
    s = warm + unroll + n_done
    g0 = s * B
    pre = tables.full_state()
    walks = eager_step(s)
    torch.cuda.synchronize(dev)
    _native.check_status(status, 'bench batch64 step check')
    n_in = int(tables._n_touched.item())                       # |U|: distinct centre rows
    n_out = int((tables.last_out[:V] == tables.step_count).sum())   # out rows stepped
    rows_in, rows_out = verify.sample_rows(walks, R, K, V, seed, g0 * per, 256)
    if os.environ.get('DW_BENCH_CORRUPT') == '1':   # test aid: the check must then fail
        tables.m_out[int(rows_out[0])] += 1e-3
    post = tables.full_state()
    gi, go = verify.sampled_grads(pre[0], pre[3], walks, R, K, seed, g0 * per, rows_in, rows_out)
    kw = dict(step=tables.step_count, lr=args.lr, betas=tables.betas, eps=tables.eps,
              weight_decay=tables.weight_decay)
    res = {'in': verify.check_rows(gi, tuple(x[rows_in] for x in pre[:3]),
                                   tuple(x[rows_in] for x in post[:3]), **kw),
           'out': verify.check_rows(go, tuple(x[rows_out] for x in pre[3:]),
                                    tuple(x[rows_out] for x in post[3:]), **kw)}
    step_check = dict(verify.summarize(res), rows_in=int(rows_in.numel()),
                      rows_out=int(rows_out.numel()), step=tables.step_count)
    del pre, post, graphed, tables
    torch.cuda.empty_cache()

    bpp = sgns_bytes_per_pair(d, K, R)
    adam_bytes = (n_in + n_out) * d * 4 * 7
    alg = pairs * bpp + adam_bytes
    gbs = alg / (kern_ms * 1e-3) / 1e9
    return {
        'workload': (f'C3 graph, the reference configs\' batch: {B} walks/step ({args.method}, '
                     f'L={L}), R={R}, K={K}, d={d}; one GPU, lazy exact Adam of both tables '
                     f'(OwnerLazyTables, rows-major out step), HIP graphs of {unroll} steps'),
        'value': pairs * n_steps / elapsed, 'unit': 'positive-pairs/s',
        'ms_per_step': elapsed / n_steps * 1e3, 'steps': n_steps, 'warmup': warm + unroll,
        'positive_pairs_per_step': pairs, 'mean_loss': mean_loss,
        'roofline': {
            'kernel': ('GraphedOwnerStep replay: Philox walker, k_out_claim + placement, '
                       'k_out_rows (rows-major out step), k_sgns_g16 centre pass, in-table '
                       'catch-up / update (k_rows_adam)'),
            'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': gbs / HBM_PEAK_GBS, 'traffic': None,
            'measured_copy_GBps': copy_gbs, 'frac_of_measured': gbs / copy_gbs,
            'ms_per_step_events': kern_ms, 'bytes_per_step': alg,
            'sgns_bytes': pairs * bpp, 'touched_rows_adam_bytes': adam_bytes,
            'touched_in_rows': n_in, 'touched_out_rows': n_out},
        'steady_state': steady,
        'step_check': step_check,
        'deterministic': bool(args.deterministic),
        'cpu_baseline': None,
    }


def c5_line(args, dev, n_walks: int, n_steps: int) -> dict:
    """BASELINE configs[4] (C5, the biased second-order walk stress config) on one GPU, timed by
    the driver's run: R-MAT 24 built on the device (16,777,216 nodes, 256M edge
    draws, 513M directed edges, hubs of 392,747 neighbours), node2vec p = .25, q = 4, L = 80.

    walks (``n_walks`` walks, one per node from node 1): the exact walker (rng='python':
    CPython's random.random() stream generated in HBM, dw_walk_replay_positions over the per-edge
    position index, built here and timed) and the Philox walker over the same index
    (dw_walk_fast_positions, layout='positions'); each with its realised bytes per step (a counted
    launch of the same walks), HBM fraction and dependent-line fraction (dependent_line_roofline).
    The index (132.6 GB) is then freed.

    step: ``n_steps`` steps of the one-GPU composition tests/test_gpu_c5_step.py checks
    (OwnerLazyTables on one rank: the in table's Adam lazy and exact, the out table's dense Adam
    fused into the records gather; d = 256, K = 5, R = 5, 8,192 Philox node2vec walks per step;
    random uniform Xavier-law init on the device), HIP-event and wall timed; roofline: SURVEY §8d's
    per-pair SGNS bytes + the out table's dense Adam (V d 28 B) + the touched in rows' (|U| d 28 B)
    over the event window. Then one more step checked from its pre-state on ~256 in and ~256 out
    rows against the float64 restatement (word2vec/verify.py, the single-step bars); a miss fails
    the bench."""
    import gc
    import random as _random
    from shallow_encoders import _native
    from shallow_encoders.graph.random_walk_generator import Node2Vec
    from shallow_encoders.graph.rmat import rmat_graph
    from shallow_encoders.graph.rng import draw_uniforms_device
    from shallow_encoders.word2vec import verify
    from shallow_encoders.word2vec.sgns import loss_terms
    from shallow_encoders.word2vec.sharding import OwnerLazyTables, owner_lazy_step
    cfg = CONFIGS['c5']
    L, p, q = cfg['walk_length'], cfg['p'], cfg['q']
    d, R, K, B = cfg['dim'], cfg['radius'], args.neg, cfg['batch_walks']
    out = {'workload': (f'C5 (BASELINE configs[4]) on one GPU: R-MAT scale {cfg["scale"]} / '
                        f'{cfg["edges"]} edge draws, node2vec p={p:g} q={q:g} L={L}; step d={d}, '
                        f'R={R}, K={K}, {B} walks/step')}
    t0 = time.perf_counter()
    csr = rmat_graph(cfg['scale'], cfg['edges'], 0, device=dev)
    V = csr.vocab_size
    torch.cuda.synchronize(dev)
    out['graph'] = {'nodes': V - 1, 'edges': csr.nnz // 2, 'build_s': time.perf_counter() - t0,
                    'max_degree': int(csr.degree().max())}
    n_walks = min(n_walks, V - 1)
    st = torch.arange(1, n_walks + 1, dtype=torch.int32, device=dev)
    walks = torch.empty((n_walks, L), dtype=torch.int32, device=dev)
    steps = n_walks * (L - 1)
    # ---- the exact walker over the position index -------------------------------------------
    torch.cuda.reset_peak_memory_stats(dev)
    a = time.perf_counter()
    dt = csr.device_tensors(dev, need_sorted=True, need_adj_pos=True, need_hub_bits=True,
                            need_edge_cn=True, need_n2v_index=True)
    torch.cuda.synchronize(dev)
    info = dict(dt.get('n2v_index_info') or {})
    out['position_index'] = dict(info, aux_and_index_build_s=time.perf_counter() - a)
    if dt.get('n2v_rec') is None:
        out['skipped'] = f'the position index does not fit this device: {info}'
        return out
    csr.philox_positions(dev)   # decided now (from the index's size: the rejection walker)
    ex = Node2Vec(csr, L, p=p, q=q, device=dev)
    _random.seed(0)
    ex.walk_batch(st[:64])                                # warm-up (jump tables)
    ex.walk_batch(st, out=walks)
    torch.cuda.synchronize(dev)
    a = time.perf_counter()
    ex.walk_batch(st, out=walks)                          # end to end from the generator state
    torch.cuda.synchronize(dev)
    e2e = time.perf_counter() - a
    u = torch.empty(steps, dtype=torch.float64, device=dev)
    draw_uniforms_device(u.numel(), dev, out=u)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    ex.walk_batch(st, uniforms=u, out=walks, check=False)
    e[1].record()
    torch.cuda.synchronize(dev)
    kern_s = e[0].elapsed_time(e[1]) * 1e-3
    c = ex.count_replay_traffic(st, u, out=walks)
    cs = max(c['steps'], 1)
    gbs = c['bytes'] / kern_s / 1e9
    out['walks_per_s_exact'] = n_walks / e2e
    out['exact_walker'] = {
        'walker': ex.last_walker, 'walks': n_walks, 'walks_per_s': n_walks / e2e,
        'kernel_walks_per_s': n_walks / kern_s, 'kernel_ms': kern_s * 1e3,
        'bytes': c['bytes'], 'bytes_per_step': c['bytes'] / cs,
        'position_units_per_step': c['entries'] / cs, 'serial_picks': c['probes'],
        'roofline': {'bound': 'dependent random lines', 'achieved': gbs, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': gbs / HBM_PEAK_GBS,
                     'random_line_roofline': dependent_line_roofline(
                         c['steps'], kern_s, 1.0 + c['lines'] / cs, info['bytes'],
                         POS_LINES)}}
    del u
    # ---- the Philox walker over the same index ------------------------------------------------
    px = Node2Vec(csr, L, p=p, q=q, rng='philox', seed=7, device=dev, layout='positions')
    px.walk_batch(st[:1024], walk_id0=0, out=walks[:1024], check=False)
    torch.cuda.synchronize(dev)
    a = time.perf_counter()
    e[0].record()
    px.walk_batch(st, walk_id0=0, out=walks)
    e[1].record()
    torch.cuda.synchronize(dev)
    e2e = time.perf_counter() - a
    kern_s = e[0].elapsed_time(e[1]) * 1e-3
    c = px.count_traffic(st, walk_id0=0, out=walks)
    cs = max(c['steps'], 1)
    gbs = c['bytes'] / kern_s / 1e9
    out['walks_per_s_philox'] = n_walks / e2e
    out['philox_walker'] = {
        'walker': px.last_walker, 'walks': n_walks, 'walks_per_s': n_walks / e2e,
        'kernel_walks_per_s': n_walks / kern_s, 'kernel_ms': kern_s * 1e3,
        'bytes': c['bytes'], 'bytes_per_step': c['bytes'] / cs,
        'position_units_per_step': c['position_loads'] / cs,
        'roofline': {'bound': 'dependent random lines', 'achieved': gbs, 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': gbs / HBM_PEAK_GBS,
                     'random_line_roofline': dependent_line_roofline(
                         c['steps'], kern_s, 1.0 + c['position_lines'] / cs, info['bytes'],
                         POS_LINES)}}
    del walks, st, ex, px
    out['hbm_peak_bytes_walks'] = torch.cuda.max_memory_allocated(dev)
    # the index and the exact walker's other structures make room for the tables
    for k in ('n2v_rec', 'n2v_pos', 'edge_cn', 'adj_hpos', 'hub_bits', 'hub_idx', 'col_sorted'):
        dt.pop(k, None)
    del dt
    gc.collect()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    # ---- the SGNS step (test_gpu_c5_step's composition) ---------------------------------------
    walker = Node2Vec(csr, L, p=p, q=q, rng='philox', seed=1234, device=dev)
    tables = OwnerLazyTables(V, d, dev, lr=args.lr, init_seed=None, emulate_world=1)
    gen = torch.Generator(device=dev).manual_seed(0)
    lim = math.sqrt(6.0 / (V + d))                        # W2VBase's Xavier law (model.py:26-27)
    tables.params_in[0, :V].uniform_(-lim, lim, generator=gen)
    tables.w_out[:V].uniform_(-lim, lim, generator=gen)
    per = L - 2 * R
    pairs = B * per * 2 * R
    grad_scale = 1.0 / pairs
    walks_total = (V - 1) * cfg['walks_per_node']
    loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    seed = 99

    def batch(s: int) -> torch.Tensor:
        g0 = s * B
        ids = (torch.arange(g0, g0 + B, device=dev, dtype=torch.int64) % walks_total) \
            // cfg['walks_per_node'] + 1
        return walker.walk_batch(ids.to(torch.int32), walk_id0=g0, check=False, status=status)

    def step(s: int, w: torch.Tensor) -> None:
        owner_lazy_step(tables, w, R, K, seed=seed, noise_offset=s * B * per,
                        grad_scale=grad_scale, loss_acc=loss_acc, status=status)

    warm = 3
    for s in range(warm):
        step(s, batch(s))
    torch.cuda.synchronize(dev)
    _native.check_status(status, 'bench c5 warmup')
    loss_acc.zero_()
    a = time.perf_counter()
    e[0].record()
    for s in range(warm, warm + n_steps):
        step(s, batch(s))
    e[1].record()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - a
    _native.check_status(status, 'bench c5')
    hbm_step = torch.cuda.max_memory_allocated(dev)   # the step's footprint (before the check)
    ev_ms = e[0].elapsed_time(e[1]) / n_steps
    mean_loss = float(loss_terms(loss_acc, pairs * n_steps, K)['loss'])
    # one more step, checked from its pre-state (the sampled rows; the tables are 17 GB each)
    s = warm + n_steps
    w = batch(s)
    rows_in, rows_out = verify.sample_rows(w, R, K, V, seed, s * B * per, 256)
    w_in = tables.w_in                                    # (flushes: every row current)
    gi, go = verify.sampled_grads(w_in, tables.w_out[:V], w, R, K, seed, s * B * per, rows_in,
                                  rows_out)
    pre_in = tuple(x[rows_in].clone() for x in (tables.params_in[0], tables.m_in, tables.v_in))
    pre_out = tuple(x[rows_out].clone() for x in (tables.w_out, tables.m_out, tables.v_out))
    step(s, w)
    torch.cuda.synchronize(dev)
    _native.check_status(status, 'bench c5 step check')
    n_in = int(tables._n_touched.item())
    tables.flush()
    if os.environ.get('DW_BENCH_CORRUPT') == '1':   # test aid: the check must then fail
        tables.m_out[int(rows_out[0])] += 1e-3
    post_in = tuple(x[rows_in] for x in (tables.params_in[0], tables.m_in, tables.v_in))
    post_out = tuple(x[rows_out] for x in (tables.w_out, tables.m_out, tables.v_out))
    kw = dict(step=tables.step_count, lr=args.lr, betas=tables.betas, eps=tables.eps,
              weight_decay=tables.weight_decay)
    res = {'in': verify.check_rows(gi, pre_in, post_in, **kw),
           'out': verify.check_rows(go, pre_out, post_out, **kw)}
    step_check = dict(verify.summarize(res), rows_in=int(rows_in.numel()),
                      rows_out=int(rows_out.numel()), step=tables.step_count)
    bpp = sgns_bytes_per_pair(d, K, R)
    out_adam, in_adam = V * d * 4 * 7, n_in * d * 4 * 7
    alg = pairs * bpp + out_adam + in_adam
    gbs = alg / (ev_ms * 1e-3) / 1e9
    out.update({
        'value': pairs * n_steps / elapsed, 'unit': 'positive-pairs/s',
        'ms_per_step': elapsed / n_steps * 1e3, 'steps': n_steps, 'warmup': warm,
        'positive_pairs_per_step': pairs, 'mean_loss': mean_loss,
        'step_composition': ('sharding.owner_lazy_step on one rank (OwnerLazyTables: lazy exact '
                             'in-table Adam, out-table dense Adam fused into the records gather); '
                             'Philox node2vec walks (rejection walker: the index is freed)'),
        'roofline': {'kernel': ('walker + k_sgns_g16<owner> + rocprim onesweep sort + '
                                'k_rec_gather with the out-table Adam fused + k_adam_rest + '
                                'touched in rows (k_rows_adam)'),
                     'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': gbs / HBM_PEAK_GBS, 'traffic': None, 'ms_per_step_events': ev_ms,
                     'bytes_per_step': alg, 'sgns_bytes': pairs * bpp,
                     'out_table_adam_bytes': out_adam, 'touched_in_rows': n_in,
                     'touched_in_rows_adam_bytes': in_adam},
        'hbm_peak_bytes_step': hbm_step,
        'step_check': step_check})
    del tables, walker, csr
    gc.collect()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=400,
                    help='timed steps (C3: ~2.7 s of GPU time, so the job clock sees the GPU busy)')
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--batch-walks', type=int, default=None)
    ap.add_argument('--config', default='c3', choices=sorted(CONFIGS),
                    help='BASELINE workload preset: c2 = Cora-shaped R-MAT 12, node2vec, 64-walk '
                         'batches; c3 = R-MAT 20 / 10M draws, d=128, DeepWalk '
                         '(the metric\'s config); c5 = R-MAT 24 / 256M draws, d=256, node2vec '
                         'p=0.25 q=4 (BASELINE configs[4], here per GPU)')
    ap.add_argument('--method', default=None, choices=['deepwalk', 'node2vec'])
    ap.add_argument('--p', type=float, default=None)
    ap.add_argument('--q', type=float, default=None)
    ap.add_argument('--scale', type=int, default=None)
    ap.add_argument('--edges', type=int, default=None)
    ap.add_argument('--dim', type=int, default=None)
    ap.add_argument('--neg', type=int, default=5)
    ap.add_argument('--radius', type=int, default=None)
    ap.add_argument('--walk-length', type=int, default=None)
    ap.add_argument('--walks-per-node', type=int, default=None)
    ap.add_argument('--lr', type=float, default=0.01)
    ap.add_argument('--scaling', default='weak', choices=['weak', 'strong'],
                    help='weak: --batch-walks walks per rank per step (the global batch grows '
                         'with N); strong: --batch-walks is the global batch, each rank trains '
                         '1/N of it (SURVEY.md §8e parity mode)')
    ap.add_argument('--scatter', default='auto', choices=['auto', 'sorted', 'atomic'],
                    help='output-table gradient: records+sort+gather (sorted) or float atomics; '
                         'auto = atomic for batches of <= 65,536 records on the one-GPU '
                         'replicated path (the C2 shape: the sort\'s launches cost more than '
                         'the atomics), sorted otherwise')
    ap.add_argument('--cpu-budget', type=float, default=20.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-walk-bench', action='store_true')
    ap.add_argument('--no-fuse-adam', action='store_true',
                    help='N=1: run the output table\'s Adam as its own pass (unfused)')
    ap.add_argument('--no-out-pieces', action='store_true',
                    help='N>1: exchange the output table after the whole output-table phase')
    ap.add_argument('--out-pieces', type=int, default=None,
                    help='N>1: output-table pieces (default sharding.DEFAULT_OUT_PIECES)')
    ap.add_argument('--no-overlap-in', action='store_true',
                    help='N=1: run the in-table Adam after the output-table phase (serial)')
    ap.add_argument('--dist-mode', default='owner', choices=['owner', 'replicated'],
                    help='N>1 layout: owner = out table sharded by row owner, every rank forms '
                         'the whole global batch and computes its own rows\' slots, only the in '
                         'table is exchanged (OwnerTables); replicated = both tables replicated, '
                         'both exchanged (ShardedTables)')
    ap.add_argument('--emulate-world', type=int, default=0,
                    help='one GPU, measurement only: run rank 0\'s share of an owner-mode job of '
                         'this many ranks (its walks, slots, Adam rows) without the collectives; '
                         'value is then a projection (comm assumed hidden)')
    ap.add_argument('--owner-walks', default='gather', choices=['all', 'gather'],
                    help='owner mode: every rank generates its own node range\'s B walks (walk '
                         'ids rank*B.., start nodes in node order) and all-gathers them over RCCL '
                         '(gather; default, north_star\'s walk sharding by node-id range), or '
                         'generates the whole global batch itself (all; a measured option)')
    ap.add_argument('--in-exchange', default=None, choices=['sharded', 'lazy', 'auto'],
                    help='owner mode, in table: sharded = dense reduce-scatter / own-rows Adam / '
                         'all-gather (OwnerTables); lazy = only the rows the batch touched are '
                         'all-reduced and updated, the others\' g = 0 Adam steps replayed exactly '
                         'when next touched (OwnerLazyTables; default at C5, where the dense '
                         'exchange is 2 x 17 GB per step); auto = time --calib-steps of each on '
                         'this job (max over ranks) before the warmup and keep the faster '
                         '(default at C3 with N > 1: which one hides better behind the '
                         'output-table phase depends on the xGMI / RCCL rate)')
    ap.add_argument('--n1-in-adam', default='auto', choices=['auto', 'dense', 'lazy'],
                    help='one GPU, in-table Adam: dense (the overlapped dense update of the fused '
                         'N=1 step) or lazy (the owner path on one rank with the lazy exact Adam: '
                         'only the rows the batch touches are read and updated, deferred g = 0 '
                         'steps replayed bit-exactly). auto = lazy when a step\'s centres are '
                         'under 10%% of the rows of a table of >= 1 GB of Adam bytes (C5: 3.4%% '
                         'of 16.8M rows; C3: 55%%, where dense measured faster)')
    ap.add_argument('--graph', default='auto', choices=['auto', 'on', 'off'],
                    help='one GPU: replay the step (replicated, or the lazy owner step) as a HIP '
                         'graph with the per-step scalars in device memory (word2vec/graphed.py); '
                         'auto = for batches of <= 100K centres, where the step is launch-bound '
                         '(the C2 shape; C3 at the reference\'s 64-walk batch)')
    ap.add_argument('--lazy-out', default='auto', choices=['auto', 'on', 'off'],
                    help='lazy in-table exchange: keep the out slice\'s Adam lazy (exact) too; '
                         'auto = when a step\'s records touch under ~half of the slice\'s rows '
                         '(C3 at 64-walk batches)')
    ap.add_argument('--layout-calib', default='auto', choices=['auto', 'on', 'off'],
                    help='N > 1, owner layout: also time --calib-steps steps of the replicated '
                         'layout (north_star\'s: node-id-range Adam shards, reduce-scatter + '
                         'all-gather = an all-reduce of both tables\' gradients) on this job, '
                         'report both (layout_calibration_ms_per_step) and run the faster; '
                         'auto = at C3 (C5\'s dense exchange is 2 x 17 GB per step)')
    ap.add_argument('--calib-steps', type=int, default=8,
                    help='--in-exchange auto: timed steps per protocol')
    ap.add_argument('--graph-unroll', type=int, default=0,
                    help='steps per captured graph (0: the largest of 16, 8, 4, 2, 1 that '
                         'divides --steps)')
    ap.add_argument('--exact-steps', type=int, default=None,
                    help='one GPU, replicated step: then time this many steps (default --steps) '
                         'with the bit-exact replay walker instead of the Philox one (rng='
                         '"python": CPython\'s random.random() stream generated in HBM from a '
                         'resident MT19937 state, dw_mt_draw, walked by dw_walk_replay(_inline)) '
                         'and report it as value_exact_walks; 0 = skip')
    ap.add_argument('--exact-prefetch', default='on', choices=['on', 'off'],
                    help='exact-walk steps: generate the next step\'s uniforms and walks on a '
                         'side stream during this step\'s SGNS')
    ap.add_argument('--verify-step', default='auto', choices=['auto', 'on', 'off'],
                    help='after the timed steps, check one more step on a sample of rows against '
                         'a float64 restatement of the reference step from the full tables '
                         '(word2vec/verify.py; every rank gathers them); exit non-zero on a miss. '
                         'auto = on for the owner layout with collectives (the N > 1 lines)')
    ap.add_argument('--walk-prefetch', action='store_true',
                    help='generate the next batch\'s walks on a side stream during this step\'s '
                         'SGNS (measured neutral on MI355X: the SGNS slows by what the walker '
                         'saves, 6.89 vs 6.89 ms/step at C3; on by default on the one-GPU lazy '
                         'path of small batches)')
    ap.add_argument('--batch64-long', type=int, default=20000,
                    help='batch64: keep replaying to this many steps and time the last 4,000 '
                         '(the in rows\' lags, and so their catch-up, grow with the run: the '
                         'steady state a reference epoch of ~163K steps runs in); 0 = skip')
    ap.add_argument('--batch64-steps', type=int, default=400,
                    help='the one-GPU C3 line: then also time this many steps at the reference '
                         'configs\' 64-walk batch (lazy exact Adam, graph-replayed) and report '
                         'them as batch64, with a checked step; 0 = skip')
    ap.add_argument('--c5-walks', type=int, default=1 << 20,
                    help='the one-GPU C3 line: then also run BASELINE configs[4] (C5) — this many '
                         'exact and Philox node2vec walks over the position index, and '
                         '--c5-steps checked SGNS steps at d=256 — reported as c5')
    ap.add_argument('--c5-steps', type=int, default=16, help='0 = skip the c5 part')
    ap.add_argument('--deterministic', action='store_true',
                    help='the deterministic accumulation mode (word2vec/exact.py: int64 '
                         'fixed-point gradient sums, bit-identical tables run to run and across '
                         'ranks); dense in-table Adam and the records path, as that mode needs')
    args = ap.parse_args()
    if args.deterministic:
        # one GPU, sparse batches keep the lazy owner path (its rows-major step has the integer
        # sums); otherwise the dense in-table Adam and the records path
        if args.n1_in_adam != 'lazy':
            args.n1_in_adam = 'auto'
        args.scatter = 'sorted'
    for k, v in CONFIGS[args.config].items():   # explicit flags override the preset
        if getattr(args, k) is None:
            setattr(args, k, v)
    if args.in_exchange is None:
        args.in_exchange = 'lazy' if args.config == 'c5' else 'auto'

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local_rank = int(os.environ.get('LOCAL_RANK', '0'))
    # rehearsal knobs (not for measurements): DW_BENCH_BACKEND=gloo and DW_BENCH_ONE_DEVICE=1
    # run N ranks on one GPU to exercise the multi-rank flow on a 1-GPU box
    backend = os.environ.get('DW_BENCH_BACKEND', 'nccl')
    if os.environ.get('DW_BENCH_ONE_DEVICE') == '1':
        local_rank = 0
    # DW_BENCH_DIST=1: take the multi-rank path (process group, collectives, owner layout) even
    # at world 1, so the RCCL flow of the N > 1 lines runs on a one-GPU box (a check, not a
    # measurement of scaling)
    dist_on = world > 1 or os.environ.get('DW_BENCH_DIST') == '1'
    if dist_on and world == 1:
        os.environ['DW_FORCE_COLLECTIVES'] = '1'   # the tables take their N > 1 protocols
    if dist_on:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local_rank)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local_rank))
        else:
            dist.init_process_group(backend)
    dev = torch.device('cuda', local_rank)
    torch.cuda.set_device(dev)
    rc = run(args, world, rank, local_rank, backend, dist_on, dev)
    line = _RESULT.pop('line', None)
    if (rc == 0 and line is not None and not dist_on and args.config == 'c3'
            and args.c5_steps > 0 and args.c5_walks > 0 and not args.deterministic
            and args.batch_walks == CONFIGS['c3']['batch_walks'] and not args.emulate_world):
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        c5 = c5_line(args, dev, args.c5_walks, args.c5_steps)
        line['c5'] = c5
        if c5.get('step_check') is not None and not c5['step_check']['ok']:
            log(rank, f'[bench] c5 step check FAILED: {c5["step_check"]}')
            rc = 3
    if line is not None and rank == 0:
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    if rc:
        sys.exit(rc)


def run(args, world: int, rank: int, local_rank: int, backend: str, dist_on: bool, dev) -> int:
    """The benchmark on this rank (process group already up when dist_on); prints the JSON line
    on rank 0 and returns the exit status (3: a step check failed). The N > 1 layout calibration
    may hand the run over to a fresh call with the faster layout."""
    from shallow_encoders import _native
    from shallow_encoders.graph.random_walk_generator import DeepWalk, Node2Vec
    from shallow_encoders.graph.rmat import rmat_graph
    from shallow_encoders.word2vec.sgns import loss_terms, phase_ms, phase_timing, sgns_phase_bytes
    from shallow_encoders.word2vec.sgns import sgns_owner_pass1, sgns_owner_pass2
    from shallow_encoders.word2vec.sharding import (OwnerLazyTables, OwnerTables, ShardedTables,
                                                    overlap_adam_blocks, owner_lazy_step,
                                                    replicated_step)
    _native.require_device(dev)

    copy_gbs = measured_copy_gbs(dev)   # before the tables take the memory
    t0 = time.time()
    csr = rmat_graph(args.scale, args.edges, 0, device=dev)   # built in HBM (dw_rmat_edges)
    V = csr.vocab_size
    N = V - 1
    log(rank, f'[bench] R-MAT scale {args.scale}: {N} nodes, {csr.nnz // 2} edges '
              f'({time.time() - t0:.1f}s)')
    csr.device_tensors(dev)
    R, K, d, L, B = args.radius, args.neg, args.dim, args.walk_length, args.batch_walks
    if args.method == 'node2vec':
        walker = Node2Vec(csr, L, p=args.p, q=args.q, rng='philox', seed=1234, device=dev)
    else:
        walker = DeepWalk(csr, L, rng='philox', seed=1234, device=dev)
    emulate = args.emulate_world if (not dist_on and args.emulate_world >= 1) else 0
    # one GPU, sparse batches: the owner path on one rank with the lazy exact in-table Adam
    # (auto: sparse batches over a large table — at C2 the table is 15 MB and the lazy path's
    # extra launches cost more than its Adam saves: 0.35 vs 0.20 ms per step)
    n1_lazy = (not dist_on and not emulate and args.dist_mode == 'owner'
               and (args.n1_in_adam == 'lazy' or
                    (args.n1_in_adam == 'auto' and B * (L - 2 * R) < 0.1 * V
                     and V * args.dim * 4 * 7 >= 1e9)))
    if n1_lazy:
        emulate, args.in_exchange = 1, 'lazy'
    owner = emulate > 0 or (dist_on and args.dist_mode == 'owner')
    if args.scatter == 'auto':
        records = B * (L - 2 * R) * 2 * R * (1 + K)
        args.scatter = 'atomic' if (not dist_on and not owner and records <= 65_536) else 'sorted'
    if owner and not (args.scatter == 'sorted' and d % 64 == 0 and d <= 512
                      and 2 * R * (1 + K) <= 64):
        raise SystemExit('owner mode needs the sorted path, d a multiple of 64 (<= 512) and '
                         '2R(1+K) <= 64; use --dist-mode replicated')
    W_eff = emulate or world            # ranks of the (possibly emulated) job
    # auto (N > 1 only; one rank has no exchange to choose): both protocols are timed below
    auto_in = owner and args.in_exchange == 'auto' and dist_on
    if owner and args.in_exchange == 'auto' and not auto_in:
        args.in_exchange = 'sharded'
    lazy = owner and args.in_exchange == 'lazy'

    def owner_tables(lazy_mode: bool):
        if not lazy_mode:
            return OwnerTables(V, d, dev, lr=args.lr, init_seed=0, emulate_world=emulate or None)
        # the out slice lazy too when a step's records touch under ~half of its rows
        rec_rank = B * W_eff * (L - 2 * R) * 2 * R * (1 + K) / W_eff
        s_rows = -(-V // W_eff)
        lazy_out = (args.lazy_out == 'on' or
                    (args.lazy_out == 'auto' and rec_rank < 0.7 * s_rows))
        return OwnerLazyTables(V, d, dev, lr=args.lr, init_seed=0, emulate_world=emulate or None,
                               lazy_out=lazy_out)

    # small batches on one GPU are replayed as a HIP graph (below); with the atomic scatter there
    # is no output-table phase for the in-table Adam to hide behind, so both tables' Adam is one
    # in-place launch after pass 1 (fewer graph nodes: no side stream, no double buffer)
    graph_small = (not dist_on and not owner and args.graph != 'off'
                   and args.method in ('deepwalk', 'node2vec') and not args.walk_prefetch
                   and (args.graph == 'on' or B * (L - 2 * R) <= 100_000))
    if owner:
        tables = owner_tables(lazy)
    else:
        tables = ShardedTables(V, d, dev, lr=args.lr, init_seed=0,
                               overlap_in=not args.no_overlap_in and not (
                                   graph_small and args.scatter == 'atomic'),
                               out_pieces=None if args.no_out_pieces else args.out_pieces)
    if args.scaling == 'strong':
        # SURVEY §8e parity mode: the global batch is --batch-walks, each rank trains 1/W of it
        if B % W_eff:
            raise SystemExit(f'--scaling strong: --batch-walks {B} must divide by {W_eff} ranks')
        B //= W_eff
    centres = B * (L - 2 * R)
    pairs_per_step = centres * 2 * R
    grad_scale = 1.0 / (pairs_per_step * W_eff)   # mean over the GLOBAL batch
    if args.deterministic:
        if auto_in or (lazy and not (n1_lazy and getattr(tables, 'lazy_out', False))):
            raise SystemExit('--deterministic needs the dense in-table exchange '
                             '(--in-exchange sharded), or one GPU\'s lazy owner path with the '
                             'lazy out table')
        tables.enable_exact(grad_scale)
    walks_total = N * args.walks_per_node
    BG = B * W_eff if owner else B      # walks each rank generates per step (owner: all ranks')
    walks_buf = torch.empty((BG, L), dtype=torch.int32, device=dev)
    starts_buf = torch.empty(BG, dtype=torch.int32, device=dev)

    # walk w of the job starts at node w // walks_per_node + 1 (the epoch's start list, resident;
    # a step's starts are a slice of it — no per-step kernels)
    from shallow_encoders.word2vec.graphed import epoch_starts_node_order
    epoch_starts = epoch_starts_node_order(N, args.walks_per_node, dev)

    def step_starts(g0: int, n: int, buf: torch.Tensor) -> torch.Tensor:
        a = g0 % walks_total
        if a + n <= walks_total:
            return epoch_starts[a:a + n]
        ids = torch.arange(a, a + n, device=dev, dtype=torch.int64) % walks_total
        torch.index_select(epoch_starts, 0, ids, out=buf[:n])
        return buf[:n]

    class WalkFeed:
        """The walks of step s, in buffer s % 2. With prefetch, step s+1's walks are generated
        on a side stream while step s's SGNS runs (the reference's DataLoader workers produce
        walks concurrently with training too); each timed step still generates exactly one
        batch. The walker is latency-bound and leaves the bandwidth to the SGNS kernels."""

        def __init__(self, n_walks, first_id, prefetch):
            nb = 2 if prefetch else 1
            self.prefetch, self.first_id = prefetch, first_id
            self.walks = [walks_buf] + [torch.empty_like(walks_buf[:n_walks])
                                        for _ in range(nb - 1)]
            self.starts = [starts_buf] + [torch.empty_like(starts_buf[:n_walks])
                                          for _ in range(nb - 1)]
            self.n = n_walks
            self.ready = [torch.cuda.Event() for _ in range(nb)]
            self.free = [None] * nb
            self.stream = torch.cuda.Stream(dev) if prefetch else None
            self.launched = -1

        def _gen(self, s):
            i = s % len(self.walks)
            g0 = self.first_id(s)
            gen_walks(step_starts(g0, self.n, self.starts[i]), g0, self.walks[i][:self.n])

        def _launch(self, s):
            i = s % 2
            with torch.cuda.stream(self.stream):
                if self.free[i] is not None:
                    self.stream.wait_event(self.free[i])
                self._gen(s)
                self.ready[i].record(self.stream)
            self.launched = s

        def get(self, s):
            """On the current stream: step s's walks."""
            if not self.prefetch:
                self._gen(s)
                return self.walks[0][:self.n]
            if self.launched < s:
                self._launch(s)
            torch.cuda.current_stream(dev).wait_event(self.ready[s % 2])
            return self.walks[s % 2][:self.n]

        def next(self, s):
            """After step s's walks are first read: start step s+1's."""
            if self.prefetch:
                self._launch(s + 1)

        def release(self, s):
            """After the last reader of step s's walks is enqueued."""
            if self.prefetch:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(dev))
                self.free[s % 2] = ev
    def philox_walks(starts, g0, out):
        walker.walk_batch(starts, walk_id0=g0, out=out, check=False)
    gen_walks = philox_walks

    loss_acc = torch.zeros(4, dtype=torch.float64, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    step_idx = [0]
    fuse = not args.no_fuse_adam and args.scatter == 'sorted' and tables.can_fuse_out_adam()
    pieces = dist_on and not args.no_out_pieces and not owner
    ev = {k: [] for k in ('walk', 'sgns', 'adam', 'gather')}
    pb = sgns_phase_bytes(B, L, R, K, d, V, args.scatter, fuse)
    p2_bytes = pb['sort'] + pb['pass2']        # the phase the in-table Adam overlaps

    def owner_one_step(record: bool):
        # every rank: the whole global batch's walks -> its own slots (pass 1) -> in-table
        # exchange on the side stream -> records sort + gather with the slice's Adam fused
        s = step_idx[0]
        step_idx[0] += 1
        g0 = s * BG                                   # global walk id of the step's batch
        # gather: this rank's B walks are global ids g0 + rank*B ... (the same global batch);
        # emulated, all W*B walks are generated here (no collective to time: conservative)
        gather = args.owner_walks == 'gather' and not emulate
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        if record:
            e[0].record()
        if gather:
            a0 = g0 + tables.rank * B
            own = walks_buf[tables.rank * B:(tables.rank + 1) * B]
            walker.walk_batch(step_starts(a0, B, starts_buf), walk_id0=a0, out=own, check=False)
            if record:
                eg = torch.cuda.Event(enable_timing=True)
                eg.record()
                ev['gather'].append((eg, e[1]))
            send = own if backend == 'nccl' else own.clone()
            dist.all_gather_into_tensor(walks_buf.view(-1), send.reshape(-1))
            walks = walks_buf
        else:
            walks = feed.get(s)
        if record:
            e[1].record()
        if lazy:
            # the lazy step as the library composes it (sharding.owner_lazy_step: on one rank the
            # rows-major out step, else catch-up -> pass 1 -> touched-row exchange -> lazy gather
            # -> touched-row update); its window is 'sgns' (no separate Adam phase)
            n_rec[0] = owner_lazy_step(tables, walks, R, K, seed=99, noise_offset=g0 * (L - 2 * R),
                                       grad_scale=grad_scale, loss_acc=loss_acc, status=status)
            if not gather:
                feed.next(s)
                feed.release(s)
            if record:
                e[2].record()
                ev['walk'].append((e[0], e[1]))
                ev['sgns'].append((e[1], e[2]))
                ev['adam'].append((e[2], e[2]))
            return
        sgns_owner_pass1(tables.w_in_raw, tables.w_out, tables.grads_in, K, walks=walks,
                         context_radius=R, owner=tables.rank, n_owners=tables.world,
                         vocab_size=V, seed=99, noise_offset=g0 * (L - 2 * R),
                         grad_scale=grad_scale, loss_acc=loss_acc, status=status)
        if not gather:
            feed.next(s)
        tables.exchange_in()        # full grid: 1/W of the in table, between RS and AG
        spec = tables.out_adam_spec() if fuse else None
        # one owner keeps every slot: no record-count readback (the host runs ahead)
        n = sgns_owner_pass2(tables.w_in_raw, tables.w_out, tables.g_out, K, walks=walks,
                             context_radius=R, out_adam=spec, status=status,
                             read_count=tables.world > 1)
        n_rec[0] = n if n is not None else BG * (L - 2 * R) * 2 * R * (1 + K)
        if not gather:
            feed.release(s)
        if spec is None:
            tables.out_step()
        if record:
            e[2].record()
        tables.sync()
        if record:
            e[3].record()
            ev['walk'].append((e[0], e[1]))
            ev['sgns'].append((e[1], e[2]))
            ev['adam'].append((e[2], e[3]))

    n_rec = [0]
    # walks: one batch per step; prefetched on a side stream unless owner 'gather' (a collective)
    # (on by default for the one-GPU lazy path, i.e. small batches: there the walker's dependent
    # chain is ~9% of a step and hides behind the previous step, 0.625 -> 0.603 ms at 64 walks)
    prefetch = (args.walk_prefetch or n1_lazy) and not (owner and args.owner_walks == 'gather'
                                                        and not emulate)
    feed = WalkFeed(BG if owner else B,
                    (lambda s: s * BG) if owner else (lambda s: (s * world + rank) * B),
                    prefetch)

    def one_step(record: bool):
        if owner:
            return owner_one_step(record)
        s = step_idx[0]
        step_idx[0] += 1
        g0 = (s * world + rank) * B                   # global walk id of this rank's batch
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if record else None
        if record:
            e[0].record()
        walks = feed.get(s)
        if record:
            e[1].record()

        def phase2_done():
            feed.release(s)
            if record:
                e[2].record()
        # pass 1 (g_in final) -> in-table Adam / exchange on a side stream while the
        # output-table phase runs (one device: the out table's Adam fused into it; N > 1: in
        # row pieces, each exchanged behind the next piece's gather) -> join
        replicated_step(tables, walks, R, K, seed=99, noise_offset=g0 * (L - 2 * R),
                        grad_scale=grad_scale, loss_acc=loss_acc, status=status,
                        scatter=args.scatter, fuse_out_adam=fuse, pieces=pieces,
                        after_pass1=lambda: feed.next(s), after_phase2=phase2_done)
        if record:
            e[3].record()
            ev['walk'].append((e[0], e[1]))
            ev['sgns'].append((e[1], e[2]))
            ev['adam'].append((e[2], e[3]))

    calib_ms = None
    if auto_in:
        # time each in-table protocol on this job (fresh tables, same init), keep the faster;
        # every rank takes the same decision from the max-over-ranks times
        calib_ms = {}
        for mode in ('sharded', 'lazy'):
            lazy = mode == 'lazy'
            del tables
            torch.cuda.empty_cache()
            tables = owner_tables(lazy)
            for _ in range(max(1, args.warmup)):
                one_step(False)
            torch.cuda.synchronize(dev)
            dist.barrier()
            a = time.perf_counter()
            for _ in range(args.calib_steps):
                one_step(False)
            torch.cuda.synchronize(dev)
            dist.barrier()
            t = torch.tensor([time.perf_counter() - a], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            calib_ms[mode] = float(t) / args.calib_steps * 1e3
        args.in_exchange = 'lazy' if calib_ms['lazy'] < calib_ms['sharded'] else 'sharded'
        lazy = args.in_exchange == 'lazy'
        del tables
        torch.cuda.empty_cache()
        tables = owner_tables(lazy)
        log(rank, f'[bench] in-table exchange calibration (ms/step): {calib_ms} -> '
                  f'{args.in_exchange}')
    # ---- north_star's layout timed beside the owner layout on this job --------
    layout_ms = getattr(args, 'layout_result', None)
    want_layout = (dist_on and owner and not emulate and args.layout_calib != 'off'
                   and (args.layout_calib == 'on' or args.config == 'c3'))
    if want_layout:
        def timed_steps(step_fn) -> float:
            for _ in range(max(1, args.warmup)):
                step_fn()
            torch.cuda.synchronize(dev)
            dist.barrier()
            a = time.perf_counter()
            for _ in range(args.calib_steps):
                step_fn()
            torch.cuda.synchronize(dev)
            dist.barrier()
            t = torch.tensor([time.perf_counter() - a], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t) / args.calib_steps * 1e3

        owner_ms = min(calib_ms.values()) if calib_ms else timed_steps(lambda: one_step(False))
        rt = ShardedTables(V, d, dev, lr=args.lr, init_seed=0,
                           out_pieces=None if args.no_out_pieces else args.out_pieces)
        r_walks = torch.empty((B, L), dtype=torch.int32, device=dev)
        r_starts = torch.empty(B, dtype=torch.int32, device=dev)
        r_acc = torch.zeros(4, dtype=torch.float64, device=dev)
        r_status = torch.zeros(1, dtype=torch.int32, device=dev)
        r_idx = [0]

        def repl_step():   # the replicated layout's step (bench.py --dist-mode replicated)
            g0 = (r_idx[0] * world + rank) * B
            r_idx[0] += 1
            walker.walk_batch(step_starts(g0, B, r_starts), walk_id0=g0, out=r_walks,
                              check=False)
            replicated_step(rt, r_walks, R, K, seed=99, noise_offset=g0 * (L - 2 * R),
                            grad_scale=1.0 / (pairs_per_step * world), loss_acc=r_acc,
                            status=r_status, scatter='sorted', fuse_out_adam=False,
                            pieces=not args.no_out_pieces)
        repl_ms = timed_steps(repl_step)
        _native.check_status(r_status, 'bench layout calibration')
        del rt, r_walks
        torch.cuda.empty_cache()
        layout_ms = {'owner': owner_ms, 'replicated': repl_ms}
        log(rank, f'[bench] layout calibration (ms/step): {layout_ms}')
        if repl_ms < owner_ms:   # north_star's layout is faster on this job: run it instead
            import copy
            del tables
            torch.cuda.empty_cache()
            a2 = copy.copy(args)
            a2.dist_mode, a2.layout_calib, a2.layout_result = 'replicated', 'off', layout_ms
            return run(a2, world, rank, local_rank, backend, dist_on, dev)
    for _ in range(args.warmup):
        one_step(False)
    torch.cuda.synchronize(dev)
    _native.check_status(status, 'bench warmup')
    # small batches on one GPU: the step replayed as a HIP graph (word2vec/graphed.py)
    graphed = None
    use_graph = graph_small and (fuse or args.scatter == 'atomic')
    # the one-GPU lazy owner step (the reference's 64-walk batch on a large graph) likewise
    graph_owner = (n1_lazy and args.graph != 'off'
                   and (args.graph == 'on' or B * (L - 2 * R) <= 100_000))
    if graph_owner:
        from shallow_encoders.word2vec.graphed import GraphedOwnerStep
        unroll = (args.graph_unroll if args.graph_unroll > 0 else
                  next(u for u in (16, 8, 4, 2, 1) if args.steps % u == 0))
        if args.steps % unroll:
            raise SystemExit(f'--graph-unroll {unroll} must divide --steps {args.steps}')
        graphed = GraphedOwnerStep(tables, walker, epoch_starts, B, R, K, seed=99,
                                   grad_scale=grad_scale, loss_acc=loss_acc, status=status,
                                   first_walk_id=step_idx[0] * BG, n_steps=args.steps + 1,
                                   unroll=unroll)
    elif use_graph:
        from shallow_encoders.word2vec.graphed import GraphedStep
        # several steps per graph: between replays the launch gap (~19 us) is as long as a
        # tiny step; the unroll divides --steps so exactly --steps steps are timed
        unroll = (args.graph_unroll if args.graph_unroll > 0 else
                  next(u for u in (16, 8, 4, 2, 1) if args.steps % u == 0))
        if args.steps % unroll:
            raise SystemExit(f'--graph-unroll {unroll} must divide --steps {args.steps}')
        graphed = GraphedStep(tables, walker, epoch_starts,
                              B, R, K, seed=99, grad_scale=grad_scale, loss_acc=loss_acc,
                              status=status, first_walk_id=step_idx[0] * B,
                              n_steps=args.steps + 1, scatter=args.scatter, unroll=unroll)
    loss_acc.zero_()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize(dev)
    phase_timing(graphed is None)
    t_start = time.perf_counter()
    if graphed is None:
        for _ in range(args.steps):
            one_step(True)
    else:
        for _ in range(args.steps // graphed.unroll):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            e[0].record()
            graphed.replay()
            e[1].record()
            ev['sgns'].append((e[0], e[1]))
            ev['walk'].append((e[0], e[0]))
            ev['adam'].append((e[1], e[1]))
    torch.cuda.synchronize(dev)
    phases = phase_ms()
    phase_timing(False)
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    _native.check_status(status, 'bench')
    # the rank's device footprint so far (tables, Adam state, CSR and walker structures,
    # workspaces: every device buffer is a torch allocation)
    hbm_peak = torch.cuda.max_memory_allocated(dev)
    kern_ms = {k: float(np.mean([a.elapsed_time(b) for a, b in v])) for k, v in ev.items() if v}
    if graphed is not None:   # one replay = `unroll` steps
        kern_ms = {k: v / graphed.unroll for k, v in kern_ms.items()}

    # ---- the same step with the bit-exact walker ----------------------------
    # rng='python': the walks the reference's DeepWalk.walk / Node2Vec.walk take from CPython's
    # random.random() stream (random_walk_generator.py:61-72,113), that stream generated in HBM
    # from a resident MT19937 state (DeviceMT, dw_mt_draw; no host round trip per step) and
    # walked by the exact replay kernels; everything else is the timed step above
    exact = None
    n_exact = args.steps if args.exact_steps is None else args.exact_steps
    if n_exact > 0 and not dist_on and not owner and graphed is None:
        import random as _random
        from shallow_encoders.graph.rng import DeviceMT
        ew = (Node2Vec(csr, L, p=args.p, q=args.q, device=dev) if args.method == 'node2vec'
              else DeepWalk(csr, L, device=dev))
        _random.seed(0)
        gen = DeviceMT.from_random(dev)
        ubufs = [torch.empty(B * (L - 1), dtype=torch.float64, device=dev) for _ in range(2)]
        ucount = [0]

        def exact_walks(starts, g0, out):
            u = ubufs[ucount[0] % 2]
            ucount[0] += 1
            gen.uniforms(u.numel(), out=u)
            ew.walk_batch(starts, uniforms=u, out=out, check=False)
        gen_walks = exact_walks
        feed = WalkFeed(B, lambda s: (s * world + rank) * B, args.exact_prefetch == 'on')
        loss_keep = loss_acc.clone()   # the headline's loss terms
        for _ in range(args.warmup):
            one_step(False)
        torch.cuda.synchronize(dev)
        for k in ev:
            ev[k].clear()
        ta = time.perf_counter()
        for _ in range(n_exact):
            one_step(True)
        torch.cuda.synchronize(dev)
        et = time.perf_counter() - ta
        _native.check_status(status, 'bench exact walks')
        loss_acc.copy_(loss_keep)
        ekern = {k: float(np.mean([a.elapsed_time(b) for a, b in v]))
                 for k, v in ev.items() if v}
        exact = {'value': pairs_per_step * n_exact / et, 'steps': n_exact,
                 'ms_per_step': et / n_exact * 1e3, 'vs_philox_step': (et / n_exact) /
                 (elapsed / args.steps), 'prefetch': args.exact_prefetch == 'on',
                 'walk_ms': ekern['walk'], 'method': args.method,
                 'walker': ('dw_mt_draw (CPython random.random() from a resident MT19937 state) '
                            '+ ' + ('dw_walk_replay_indexed' if args.method == 'node2vec'
                                    else 'dw_walk_replay_inline'))}

    # ---- one more step, checked on a sample of rows ---------------------------
    # every rank gathers the full tables before and after it; rank 0 restates the step in float64
    # for ~256 in rows and ~256 out rows and holds them to the single-step bars. DW_BENCH_CORRUPT=1
    # perturbs one sampled out row in the last rank's shard after the step: the check must fail.
    step_check = None
    want_check = (args.verify_step == 'on' or
                  (args.verify_step == 'auto' and dist_on))
    if want_check and (owner or dist_on) and not emulate and graphed is None and \
            (not owner or args.owner_walks == 'gather') and V * d * 4 * 6 <= (16 << 30):
        from shallow_encoders.word2vec import verify
        loss_keep = loss_acc.clone()
        # the checked step's global batch: owner — every rank's walks_buf; replicated — rank r's
        # B walks are global ids (s * world + r) * B.., gathered in rank order below
        g0 = step_idx[0] * (BG if owner else world * B)
        pre = tables.full_state()
        one_step(False)
        torch.cuda.synchronize(dev)
        _native.check_status(status, 'bench step check')
        if owner:
            walks_chk = walks_buf.clone()
        else:
            mine = feed.walks[0][:B].contiguous()
            walks_chk = torch.empty((world * B, L), dtype=torch.int32, device=dev)
            if dist_on:
                if backend == 'nccl':
                    dist.all_gather_into_tensor(walks_chk.view(-1), mine.view(-1))
                else:
                    dist.all_gather(list(walks_chk.view(world, B, L).unbind(0)), mine.clone())
            else:
                walks_chk.copy_(mine)
        rows_in, rows_out = verify.sample_rows(walks_chk, R, K, V, 99, g0 * (L - 2 * R), 256)
        if os.environ.get('DW_BENCH_CORRUPT') == '1' and tables.rank == tables.world - 1:
            if owner:
                bad = rows_out[rows_out % tables.world == tables.rank][0]
                tables.m_out[int(bad) // tables.world] += 1e-3   # a corrupted shard row
            else:   # an out row whose Adam state this rank holds
                mine_rows = tables.state_rows(1).to(dev)
                hit = torch.nonzero(torch.isin(mine_rows, rows_out)).flatten()
                tables.m[1][int(hit[0])] += 1e-3
        post = tables.full_state()
        loss_acc.copy_(loss_keep)
        if rank == 0:
            gi, go = verify.sampled_grads(pre[0], pre[3], walks_chk, R, K, 99, g0 * (L - 2 * R),
                                          rows_in, rows_out)
            kw = dict(step=tables.step_count, lr=args.lr, betas=tables.betas, eps=tables.eps,
                      weight_decay=tables.weight_decay)
            res = {'in': verify.check_rows(gi, tuple(x[rows_in] for x in pre[:3]),
                                           tuple(x[rows_in] for x in post[:3]), **kw),
                   'out': verify.check_rows(go, tuple(x[rows_out] for x in pre[3:]),
                                            tuple(x[rows_out] for x in post[3:]), **kw)}
            step_check = dict(verify.summarize(res), rows_in=int(rows_in.numel()),
                              rows_out=int(rows_out.numel()), step=tables.step_count)
        del pre, post
        torch.cuda.empty_cache()
    if owner and dist_on:               # each rank summed the loss terms of its own slots
        dist.all_reduce(loss_acc)
    terms = loss_terms(loss_acc, pairs_per_step * args.steps * (W_eff if owner else 1), K)
    mean_loss = None if emulate > 1 else float(terms['loss'])   # one rank owns every slot at W=1

    # weak scaling: the job processes B walks per rank per step (owner: W*B walks, each rank a
    # 1/W share of their slots)
    total_pairs = pairs_per_step * args.steps * W_eff
    value = total_pairs / elapsed
    bpp = sgns_bytes_per_pair(d, K, R)
    sgns_ms = phases['pass1'] + phases['sort'] + phases['pass2']
    # algorithmic bytes of the timed op: SURVEY §8d's per-pair SGNS figure, plus its dense-Adam
    # figure for one table (V*d*4 B x 7) when the out table's Adam is fused into pass 2
    out_adam_bytes = V * d * 4 * 7 if fuse else 0
    # one GPU, overlap_in: the in-table Adam (the other V*d*4 B x 7) runs on a side stream
    # inside the output-table phase; the window then ends when both streams are done
    overlap_in = not dist_on and not owner and tables.overlap_in
    in_adam_bytes = V * d * 4 * 7 if overlap_in else 0
    op_ms = sgns_ms + (kern_ms['adam'] if overlap_in else 0.0)
    if graphed is not None:     # one replay: walk + SGNS + both tables' Adam
        op_ms = kern_ms['sgns']
        out_adam_bytes = in_adam_bytes = V * d * 4 * 7
    if owner:
        # this rank's share of the job's algorithmic bytes: 1/W of the pairs' SGNS bytes and of
        # both tables' dense Adam (out slice fused in pass 2, own in-table rows on the side
        # stream); the window runs to the end of the in-table update
        out_adam_bytes = V * d * 4 * 7 // W_eff
        in_adam_bytes = V * d * 4 * 7 // W_eff
        op_ms = sgns_ms + kern_ms['adam']
        if lazy:   # + the centre order, touched-row catch-up and gather outside the pass events
            op_ms = kern_ms['sgns'] + kern_ms['adam']
            # the lazy exact Adam needs the dense figure only on the rows the batch touches
            # (every rank updates all of them); the last step's |U| stands for the steps
            in_adam_bytes = int(tables._n_host[0]) * d * 4 * 7
            if tables.lazy_out:   # the out slice's rows its records touch (expected count)
                out_adam_bytes = int(tables.S * -math.expm1(-n_rec[0] / tables.S)) * d * 4 * 7
    sgns_gbs = (pairs_per_step * bpp + out_adam_bytes + in_adam_bytes) / (op_ms * 1e-3) / 1e9
    phase_bytes = sgns_phase_bytes(B, L, R, K, d, V, args.scatter, fuse)
    if owner:
        # implementation byte model of one rank's owner passes: every centre of the global
        # batch reads its in row and adds its partial gradient row; n_rec owned slots each
        # gather an out row (pass 1) and a centre row (pass 2) with 12-B records; the slice Adam
        c_all, rows4 = BG * (L - 2 * R), 4 * d
        bits = max(1, math.ceil(math.log2(tables.S)))
        phase_bytes = {'pass1': c_all * 2 * rows4 + n_rec[0] * (rows4 + 12) + BG * L * 4,
                       'sort': n_rec[0] * (4 + 24 * math.ceil(bits / 11)),
                       'pass2': n_rec[0] * (12 + rows4) + tables.S * d * 24}
    phase_info = {k: {'ms': phases[k], 'bytes_model': phase_bytes[k],
                      'GBps': phase_bytes[k] / (phases[k] * 1e-3) / 1e9 if phases[k] else None}
                  for k in ('pass1', 'sort', 'pass2')}

    # ---- walker alone: walks/s, roofline, and the bit-exact replay walker ---------------------
    p2, q2 = (args.p, args.q) if args.method == 'node2vec' else (0.25, 4.0)
    walk_methods = (('deepwalk', 1.0, 1.0), ('node2vec', p2, q2))
    walk_stats, walk_roof, replay_stats = {}, {}, {}
    line_rate = walk_line_rates(csr.nnz * 16)
    if not args.no_walk_bench:
        # one walk per node (N walks) for both: a sample far beyond the ~50K walkers the chip
        # keeps in flight, so no partial last round of walkers skews the rate
        for meth, p, q in walk_methods:
            n_walks = N
            w = (Node2Vec(csr, L, p=p, q=q, rng='philox', seed=7, device=dev)
                 if meth == 'node2vec' else DeepWalk(csr, L, rng='philox', seed=7, device=dev))
            st = torch.arange(1, n_walks + 1, dtype=torch.int32, device=dev)
            out = torch.empty((n_walks, L), dtype=torch.int32, device=dev)
            w.walk_batch(st[:1024], walk_id0=0, out=out[:1024], check=False)
            if dist_on:
                dist.barrier()
            torch.cuda.synchronize(dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a = time.perf_counter()
            e0.record()
            w.walk_batch(st, walk_id0=rank * n_walks, out=out, check=False)
            e1.record()
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - a
            kern_s = e0.elapsed_time(e1) * 1e-3
            if dist_on:
                t = torch.tensor([dt], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt = float(t)
            walk_stats[meth] = n_walks * world / dt
            steps = n_walks * (L - 1)
            if meth == 'deepwalk':
                # the edge-inline walker: the start's row_ptr pair, one 16-B entry per step
                # (+ prob_thr / alias on weighted graphs), the walk's L int32 ids
                per_step = 16 + (8 if csr.weights is not None else 0)
                nbytes = n_walks * (16 + (L - 1) * per_step + 4 * L)
                extra = {'bytes_per_step': per_step + 4.0, 'dependent_loads_per_step': 1}
                if line_rate:
                    extra['random_line_roofline'] = {
                        'steps_per_s': steps / kern_s,
                        'chase_lines_per_s': line_rate['chase_lines_per_s'],
                        'gather_lines_per_s': line_rate['gather_lines_per_s'],
                        'frac_of_chase': steps / kern_s / line_rate['chase_lines_per_s'],
                        'frac_of_gather': steps / kern_s / line_rate['gather_lines_per_s'],
                        'source': line_rate['source']}
            else:
                # realised traffic of the same walks (dw_walk_fast_counted, untimed launch)
                c = w.count_traffic(st, walk_id0=rank * n_walks, out=out)
                nbytes = c['bytes']
                cs = max(c['steps'], 1)
                extra = {'bytes_per_step': c['bytes'] / cs,
                         'proposal_blocks_per_step': c['blocks'] / cs,
                         'adjacency_tests_per_step': c['tests'] / cs,
                         'walker': w.last_walker}
                info = csr.device_tensors(dev).get('n2v_index_info') or {}
                if 'position_loads' in c:
                    # over the position index: the step's 32-B edge record (one line), then the
                    # pick's binary-search probes, each a dependent 2-B load (C3's lists are
                    # uint16: one probe per unit)
                    extra['position_loads_per_step'] = c['position_loads'] / cs
                    extra['random_line_roofline'] = dependent_line_roofline(
                        steps, kern_s, 1.0 + c['position_lines'] / cs,
                        int(info.get('bytes') or csr.nnz * 32), POS_LINES)
                else:
                    # rejection: the row pair, a line per proposal block, a bucket per test
                    extra['random_line_roofline'] = dependent_line_roofline(
                        steps, kern_s, 1.0 + (c['blocks'] + c['tests']) / cs, csr.nnz * 4,
                        'row pair + proposal blocks + hash buckets')
            gbs = nbytes / kern_s / 1e9
            walk_roof[meth] = dict({'kernel_ms': kern_s * 1e3, 'walks': n_walks, 'bytes': nbytes,
                                    'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                    'frac': gbs / HBM_PEAK_GBS, 'p': p, 'q': q}, **extra)
            del out
        # the reference-exact walker (rng='python', dw_walk_replay): CPython's random.random()
        # stream, generated in HBM from the global generator's state (dw_mt_uniforms; the state
        # is handed back), fp64 choices arithmetic. Unweighted graphs take the exact
        # margin-checked picks (no serial sums; the serial replay only where the margin fails).
        # walks_per_s: end to end from the generator's state (stream generation, the walk, the
        # state copied back, the status check); kernel_walks_per_s: the walk alone (uniforms
        # already in HBM, HIP events); uniforms_ms: dw_mt_uniforms alone; walks_per_s_host_uniforms:
        # the previous path (numpy draws on the host + their 8 B per step copied in)
        if rank == 0 and not dist_on:
            import random as _random
            from shallow_encoders.graph.rng import draw_uniforms, draw_uniforms_device
            for meth, p, q in walk_methods:
                n_r = N   # one walk per node (the reference's epoch: a walk from every node)
                w = (Node2Vec(csr, L, p=p, q=q, device=dev) if meth == 'node2vec'
                     else DeepWalk(csr, L, device=dev))
                st = (torch.arange(n_r, dtype=torch.int32) % N) + 1   # node ids 1..N, cycled
                st_dev = st.to(dev)
                out = torch.empty((n_r, L), dtype=torch.int32, device=dev)
                build_ms = None
                if meth == 'node2vec':   # the per-edge class counts, built once per graph (timed)
                    csr.device_tensors(dev, need_sorted=True, need_adj_pos=True,
                                       need_hub_bits=True)
                    torch.cuda.synchronize(dev)
                    a = time.perf_counter()
                    csr.device_tensors(dev, need_edge_cn=True)
                    torch.cuda.synchronize(dev)
                    build_ms = (time.perf_counter() - a) * 1e3
                    # the position index (dw_n2v_edge_index_build), built once per graph (timed
                    # inside the build; entries and bytes reported)
                    csr.device_tensors(dev, need_n2v_index=True)
                _random.seed(0)
                w.walk_batch(st_dev[:64])                              # warm-up (jump tables)
                w.walk_batch(st_dev, out=out)
                torch.cuda.synchronize(dev)
                a = time.perf_counter()
                w.walk_batch(st_dev, out=out)
                torch.cuda.synchronize(dev)
                dt = time.perf_counter() - a
                u_dev = torch.empty(n_r * (L - 1), dtype=torch.float64, device=dev)
                e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                e[0].record()
                draw_uniforms_device(u_dev.numel(), dev, out=u_dev, defer=True)[1]()
                e[1].record()
                e[2].record()
                w.walk_batch(st_dev, uniforms=u_dev, out=out, check=False)
                e[3].record()
                torch.cuda.synchronize(dev)
                gen_s = e[0].elapsed_time(e[1]) * 1e-3
                kern_s = e[2].elapsed_time(e[3]) * 1e-3
                gen = _random.Random(0)
                u = draw_uniforms(n_r * (L - 1), gen)
                torch.cuda.synchronize(dev)
                a = time.perf_counter()
                w.walk_batch(st, uniforms=u, out=out)
                torch.cuda.synchronize(dev)
                dt_host = time.perf_counter() - a
                replay_stats[meth] = {'walks': n_r, 'p': p, 'q': q, 'walks_per_s': n_r / dt,
                                      'kernel_walks_per_s': n_r / kern_s,
                                      'kernel_ms': kern_s * 1e3, 'uniforms_ms': gen_s * 1e3,
                                      'uniforms_GBps': u_dev.numel() * 8 / gen_s / 1e9,
                                      'walks_per_s_host_uniforms': n_r / dt_host}
                if build_ms is not None:
                    replay_stats[meth]['edge_counts_build_ms'] = build_ms
                    info = csr.device_tensors(dev).get('n2v_index_info', {})
                    replay_stats[meth]['position_index'] = dict(info)
                    replay_stats[meth]['walker'] = (
                        'dw_walk_replay_positions (lane per walker over the position index)'
                        if csr.device_tensors(dev).get('n2v_rec') is not None
                        else 'dw_walk_replay_indexed (wave per walker, per-edge counts)')
                if meth == 'node2vec':
                    # the bit-exact walker's realised traffic (counted launch, same walks,
                    # untimed: the position walker's 32-B edge record, uniform and output per
                    # step and 4 B per position read; the wave walker's row pairs, list entries
                    # and 64-B hash buckets for the steps handed to it)
                    c = w.count_replay_traffic(st_dev, u_dev, out=out)
                    gbs = c['bytes'] / kern_s / 1e9
                    walk_roof['node2vec_replay'] = {
                        'kernel_ms': kern_s * 1e3, 'walks': n_r, 'bytes': c['bytes'],
                        'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                        'frac': gbs / HBM_PEAK_GBS, 'p': p, 'q': q,
                        'bytes_per_step': c['bytes'] / max(c['steps'], 1),
                        'hash_probes_per_step': c['probes'] / max(c['steps'], 1),
                        'list_entries_per_step': c['entries'] / max(c['steps'], 1),
                        'walker': w.last_walker}
                    if w.last_walker == 'dw_walk_replay_positions':
                        # one lane per walker: the 32-B edge record, then the exact pick's
                        # dependent position probes (2-B units; the rare serial picks' run
                        # loads counted with them); the step's uniform is an independent load
                        info = csr.device_tensors(dev).get('n2v_index_info') or {}
                        walk_roof['node2vec_replay']['random_line_roofline'] = \
                            dependent_line_roofline(
                                c['steps'], kern_s, 1.0 + c['lines'] / max(c['steps'], 1),
                                int(info.get('bytes') or csr.nnz * 32), POS_LINES)
                del out, u_dev, u

    result = {
        'metric': 'positive-pairs/s + random-walks/s, 1M-node d=128 k=5, 1/2/4/8 MI355X',
        'value': value,
        'unit': 'positive-pairs/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'ms_per_step': elapsed / args.steps * 1e3,
        'higher_is_better': True,
        'scaling': args.scaling,
        'vs_baseline': None,
        'dtype': 'fp32',
        'data': f'synthetic (R-MAT scale {args.scale} graph built on the device, Philox walks, '
                f'uniform device negatives, random Xavier init)',
        'config': {
            'workload': (f'{args.config.upper()}: R-MAT {N} nodes / {csr.nnz // 2} edges, '
                         f'{args.method}{f" p={args.p} q={args.q}" if args.method == "node2vec" else ""} L={L}, '
                         f'R={R}, K={K}, d={d}, dense Adam; {B} walks/step/GPU; '
                         f'{args.scatter} output-table scatter'),
            'global_batch_walks': B * W_eff, 'positive_pairs_per_step_per_gpu': pairs_per_step,
            'parallelism': (
                'dp1 (one GPU; owner path on one rank with the lazy exact in-table Adam: only '
                'the rows the batch touches are read and updated, deferred g = 0 steps replayed '
                'bit-exactly)' if n1_lazy else
                f'EMULATED rank 0 of {W_eff} on one GPU (owner-computes, in table '
                f'{args.in_exchange}; no collectives run, '
                f'value is a projection assuming the in-table exchange stays hidden; walks: '
                f'{args.owner_walks})' if emulate
                else f'REHEARSAL dp{world} over {backend}, all ranks on one device'
                if backend != 'nccl' and dist_on else
                f'dp{world} owner-computes (out table sharded by row owner o % {world}, no '
                f'out-table collective; in table replicated: '
                + ('touched rows all-reduced over RCCL, lazy exact Adam' if lazy else
                   'RCCL reduce-scatter / all-gather')
                + f' overlapped with the output-table phase; walks: {args.owner_walks})' if owner
                else
                f'dp{world} (node-id-range sharded Adam, RCCL reduce-scatter/all-gather, '
                f'in-table exchange overlapped'
                + (f', out table in {tables.P} pieces pipelined' if pieces else '') + ')'),
        },
        'layout': args.dist_mode if dist_on else None,
        'layout_calibration_ms_per_step': layout_ms,
        'deterministic': bool(args.deterministic),
        'in_exchange': args.in_exchange if owner else None,
        'in_exchange_calibration_ms_per_step': calib_ms,
        'walks_per_s': walk_stats.get('deepwalk'),
        f'walks_per_s_node2vec_p{p2:g}_q{q2:g}': walk_stats.get('node2vec'),
        'roofline_walk': walk_roof or None,
        'walks_per_s_replay': replay_stats or None,
        'kernel_ms': kern_ms,
        'records_per_step_per_gpu': n_rec[0] if owner else pairs_per_step * (1 + K),
        'mean_loss': mean_loss,
        'rccl_world': dist.get_world_size() if dist_on else None,
        'exposed_collective_ms_per_step': ({
            'walks_allgather': kern_ms.get('gather'),
            'after_output_phase': kern_ms.get('adam'),
            'note': ('walks_allgather: the all-gather of the node-range walks (main stream); '
                     'after_output_phase: from the end of the output-table phase to the in '
                     'table being current (the exchange not hidden behind sort + pass 2, plus the '
                     'touched-row update in the lazy exchange)')} if owner and dist_on else None),
        'step_check': step_check,
        'value_exact_walks': exact['value'] if exact else None,
        'exact_walks': exact,
        'roofline': {
            'kernel': ('dw_sgns_owner_pass1 + dw_sgns_owner_pass2 = k_sgns_g16<owner> + rocprim '
                       'onesweep radix sort + k_rec_gather with the out-slice Adam fused + '
                       'k_adam_rest || own in-table rows: reduce-scatter, k_adam, all-gather '
                       '(side stream)') if owner else
                      (('dw_sgns_walks_phase 1 + dw_sgns_walks_phase2_adam = k_sgns_g16 + rocprim '
                        'onesweep radix sort + k_rec_gather with the out-table Adam fused + '
                        'k_adam_rest' + (' || in-table k_adam (dw_adam_dense_to, side stream)'
                                         if overlap_in else '')) if fuse else
                       'dw_sgns_walks = k_sgns_g16 + rocprim onesweep radix sort + k_rec_gather'
                       if args.scatter == 'sorted' else 'dw_sgns_walks (k_sgns, atomic scatter)'),
            'bound': 'hbm', 'achieved': sgns_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': sgns_gbs / HBM_PEAK_GBS, 'traffic': None,
            'measured_copy_GBps': copy_gbs, 'frac_of_measured': sgns_gbs / copy_gbs,
            'bytes_per_pair': bpp, 'pairs_per_launch': pairs_per_step,
            'out_table_adam_bytes': out_adam_bytes, 'in_table_adam_bytes': in_adam_bytes,
            'in_table_adam_blocks': (overlap_adam_blocks(V * d * 4 * 7, p2_bytes)
                                     if overlap_in else None),
            'ms_per_launch': op_ms,
            'launches_timed': (phases['calls'] if graphed is None
                               else args.steps // graphed.unroll),
            'graph': (None if graphed is None else
                      f'HIP graph replay of walk + SGNS + both Adams (word2vec/graphed.py), '
                      f'{graphed.unroll} steps per graph; ms_per_launch is per step, the '
                      f'window is the whole replay, phases are not split'),
            'phases': phase_info,
        },
        'cpu_baseline': None,
        'hbm_peak_bytes': hbm_peak,
    }
    prof = os.path.join(REPO, 'profiles', 'sgns_pmc.json')
    if os.path.exists(prof):
        try:
            with open(prof) as f:
                doc = json.load(f)
            # (owner form: its own in-table rows' Adam runs on the side stream inside the op)
            want = (pairs_per_step, args.scatter, d, V, fuse, overlap_in or owner,
                    W_eff if owner else 0, args.in_exchange if owner else None)
            pmc = next((e for e in reversed(doc.get('entries', [])) if   # the latest round
                        (e.get('pairs_per_launch'), e.get('scatter'), e.get('dim'),
                         e.get('vocab_size'), bool(e.get('fused_out_adam')),
                         bool(e.get('overlap_in')), int(e.get('owner_world') or 0),
                         e.get('in_exchange')) == want),
                       None)
            if pmc is not None:
                result['roofline']['traffic'] = pmc.get('hbm_bytes_per_launch')
                result['roofline']['traffic_source'] = f"profiles/sgns_pmc.json ({pmc.get('round')})"
                per_k = pmc.get('hbm_bytes_per_kernel') or {}
                for k in ('pass1', 'sort', 'pass2'):
                    result['roofline']['phases'][k]['traffic'] = per_k.get('sgns_' + k)
        except (OSError, ValueError):
            pass
    # ---- the reference configs' own 64-walk batch on the same graph ---------
    b64 = None
    if (args.batch64_steps > 0 and not dist_on and not owner and not emulate
            and args.config == 'c3' and B != 64):
        del tables
        torch.cuda.empty_cache()
        b64 = batch64_line(csr, args, dev, epoch_starts, copy_gbs, args.batch64_steps)
        prof64 = os.path.join(REPO, 'profiles', 'sgns_pmc.json')
        try:
            with open(prof64) as f:
                ent = [e for e in json.load(f).get('entries', [])
                       if e.get('workload') == 'c3_batch64']
            if ent:
                b64['roofline']['traffic'] = ent[-1].get('hbm_bytes_per_launch')
                b64['roofline']['traffic_source'] = f"profiles/sgns_pmc.json ({ent[-1].get('round')})"
        except (OSError, ValueError):
            pass
        result['batch64'] = b64
    if rank == 0 and not dist_on and not args.no_cpu_baseline and args.config in ('c2', 'c3'):
        cb = cpu_baseline(csr, args, args.cpu_budget, walk_methods)
        result['cpu_baseline'] = cb
        if b64 is not None:
            s64 = next(x for x in cb['batches'] if x['batch_walks'] == 64)
            b64['cpu_baseline'] = {
                'value': s64['pairs_per_s'], 'unit': 'positive-pairs/s', 'cores': cb['cores'],
                'kind': 'port', 'sample': (f'the oracle SGNS step at 64 walks/step ({s64["steps"]} '
                                           f'steps, {s64["seconds"]:.1f}s; see cpu_baseline)')}
    if rank == 0:   # printed by main (after the c5 part)
        _RESULT['line'] = result
    failed = bool(step_check) and not step_check['ok']
    if b64 is not None and not b64['step_check']['ok']:
        log(rank, f'[bench] batch64 step check FAILED: {b64["step_check"]}')
        failed = True
    if dist_on:
        flag = torch.tensor([1 if failed else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)   # every rank exits with rank 0's verdict
        failed = bool(flag.item())
    if failed:
        log(rank, f'[bench] step check FAILED: {step_check}')
        return 3
    return 0


if __name__ == '__main__':
    main()
