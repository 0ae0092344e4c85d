"""Generate the golden fixtures from the REFERENCE itself (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [downstream | cbow | cora | traj128 | hubs]

Imports the importable pieces of /root/reference: the walkers
(graph/random_walk_generator.py), the datasets (graph/datasets.py), SkipGram (word2vec/model.py),
NegativeSamplingLoss (word2vec/loss.py) and generate_noise_batch (word2vec/utils/sampling.py),
plus torch.optim.Adam / StepLR — and records their outputs as small .npz files next to this
script. The reference's trainer / collate / config modules need pytorch_lightning, torchtext
and hydra (absent), so the training-step wiring below restates trainer.py:131-152 and the sg
collate rule (torch_dataset.py:300-309) around the reference's own model / loss / sampler.

The reference package is named ``shallow_encoders`` like the product, so the product is never
imported here; the R-MAT edge list comes from the product generator in a child process.
Nothing written here is read from /root/reference at test time.
"""
import json
import os
import random
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'

sys.dont_write_bytecode = True
sys.path.insert(0, REF)

import networkx as nx  # noqa: E402
import torch  # noqa: E402

from shallow_encoders.graph import datasets as ref_ds  # noqa: E402
from shallow_encoders.graph import random_walk_generator as ref_rwg  # noqa: E402
from shallow_encoders.word2vec.loss import NegativeSamplingLoss  # noqa: E402
from shallow_encoders.word2vec.model import SkipGram  # noqa: E402
from shallow_encoders.word2vec.utils.sampling import generate_noise_batch  # noqa: E402

assert os.path.realpath(ref_rwg.__file__).startswith(REF), 'must import the reference'


# ------------------------------------------------------------------------------- helpers
def vocab_of(graph):
    """torchtext rule for graphs (torch_dataset.py:98-110): <unk>, then sorted tokens."""
    names = [str(n) for n in graph]
    itos = ['<unk>'] + sorted(n.lower() for n in names)
    stoi = {t: i for i, t in enumerate(itos)}
    return itos, stoi


def csr_of(graph, stoi):
    """CSR in vocab space, rows in graph.neighbors() order (written independently of the
    product's builder so that it pins it)."""
    V = len(stoi)
    rows = [[] for _ in range(V)]
    wrows = [[] for _ in range(V)]
    weighted = nx.is_weighted(graph)
    for n in graph:
        i = stoi[str(n).lower()]
        for x in graph.neighbors(n):
            rows[i].append(stoi[str(x).lower()])
            if weighted:
                wrows[i].append(float(graph[n][x]['weight']))
    row_ptr = np.zeros(V + 1, dtype=np.int64)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.array([c for r in rows for c in r], dtype=np.int32)
    w = np.array([c for r in wrows for c in r], dtype=np.float64) if weighted else np.zeros(0)
    return row_ptr, col, w, weighted


class Capture:
    """Records every random.random() the reference consumes and every random.choices call."""

    def __init__(self):
        self.uniforms = []
        self.choices = []
        self._orig_random = random._inst.random
        self._orig_choices = random.choices

    def __enter__(self):
        def rec():
            u = self._orig_random()
            self.uniforms.append(u)
            return u

        def choices(population, weights=None, *, cum_weights=None, k=1):
            self.choices.append((list(population), list(weights)))
            return self._orig_choices(population, weights=weights, cum_weights=cum_weights, k=k)

        random._inst.random = rec
        random.choices = choices
        return self

    def __exit__(self, *exc):
        del random._inst.random
        random.choices = self._orig_choices
        return False


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f'wrote {path} ({os.path.getsize(path)} bytes)')


# ------------------------------------------------------------------------------- walks
def dataset_fixture(name, ds_cls, seed, walks_per_node, walk_length, method, method_params=None,
                    extra=None):
    """F1/F2/F4: one epoch of RandomWalkDataset iteration under random.seed(seed). ``extra``:
    more arrays to store, or a function of the dataset returning them."""
    random.seed(seed)
    kwargs = dict(walks_per_node=walks_per_node, walk_length=walk_length, method=method)
    if method_params is not None:
        kwargs['method_params'] = method_params
    ds = ds_cls(**kwargs)
    itos, stoi = vocab_of(ds.graph)
    row_ptr, col, w, weighted = csr_of(ds.graph, stoi)
    order = np.array([stoi[str(n).lower()] for n in ds._nodes], dtype=np.int32)
    with Capture() as cap:
        walks = [s.split() for s in ds]          # full epoch; StopIteration reshuffles
    order_after = np.array([stoi[str(n).lower()] for n in ds._nodes], dtype=np.int32)
    ids = np.array([[stoi[t.lower()] for t in wk] for wk in walks], dtype=np.int32)
    L = walk_length
    u = np.array(cap.uniforms, dtype=np.float64).reshape(len(walks), max(L - 1, 0))
    # per-step normalised weights as passed to random.choices (the reference transition law)
    pops = [np.array([stoi[str(x).lower()] for x in pop], dtype=np.int32) for pop, _ in cap.choices]
    wts = [np.array(wt, dtype=np.float64) for _, wt in cap.choices]
    offs = np.zeros(len(pops) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(p) for p in pops])
    p = q = 1.0
    if method_params:
        p, q = float(method_params.get('p', 1.0)), float(method_params.get('q', 1.0))
    more = extra(ds) if callable(extra) else (extra or {})
    save(name, **more, seed=seed, walks_per_node=walks_per_node, walk_length=L,
         method=np.array(method), p=p, q=q, itos=np.array(itos), row_ptr=row_ptr, col=col,
         weights=w, weighted=weighted, order=order, order_after=order_after,
         starts=ids[:, 0].copy(), uniforms=u, walks=ids,
         step_pop=np.concatenate(pops) if pops else np.zeros(0, np.int32),
         step_w=np.concatenate(wts) if wts else np.zeros(0), step_off=offs)


def rmat_fixture(name, scale, n_edges, graph_seed, seed, n_walks, walk_length, method, p=1.0,
                 q=1.0):
    """F3: reference walker on the R-MAT graph (edges from the product generator)."""
    tmp = os.path.join(HERE, f'_edges_{scale}_{n_edges}_{graph_seed}.npy')
    code = (f"import sys; sys.path.insert(0, {os.path.join(REPO, 'deepwalk-and-node2vec_amd')!r});"
            f"import numpy as np; from shallow_encoders.graph.rmat import rmat_edges;"
            f"e, _ = rmat_edges({scale}, {n_edges}, {graph_seed}); np.save({tmp!r}, e)")
    subprocess.run([sys.executable, '-c', code], check=True,
                   env=dict(os.environ, PYTHONDONTWRITEBYTECODE='1'))
    edges = np.load(tmp)
    os.remove(tmp)
    n = 1 << scale
    g = nx.Graph()
    g.add_edges_from((f'n{u:07d}', f'n{v:07d}') for u, v in edges.tolist())
    itos, stoi = vocab_of(g)
    assert len(itos) == n + 1
    row_ptr, col, w, weighted = csr_of(g, stoi)
    rng = np.random.default_rng(seed)
    starts = rng.integers(1, n + 1, size=n_walks).astype(np.int32)
    params = {'p': p, 'q': q} if method == 'node2vec' else None
    walker = ref_rwg.random_walk_factory(method, g, walk_length, params)
    random.seed(seed)
    walks = []
    with Capture() as cap:
        for s in starts:
            walks.append([stoi[t.lower()] for t in walker.walk(itos[s]).split()])
    u = np.array(cap.uniforms, dtype=np.float64).reshape(n_walks, walk_length - 1)
    save(name, scale=scale, n_edges=n_edges, graph_seed=graph_seed, seed=seed,
         walk_length=walk_length, method=np.array(method), p=p, q=q, edges=edges.astype(np.int32),
         row_ptr=row_ptr, col=col, starts=starts, uniforms=u,
         walks=np.array(walks, dtype=np.int32))


def hub_fixture(name, scale, n_edges, graph_seed, seed, method, p=1.0, q=1.0, n_hubs=8,
                walks_per_hub=3, walk_length=8):
    """the reference walker from the top-degree nodes of a large R-MAT graph
    (R-MAT 20 = C3's graph: hubs up to 44,848 neighbours), so the replay kernel's exact picks
    are pinned by the reference itself at hub rows far beyond LDS. The graph is not stored
    (80 MB): the fixture keeps its spec and SHA-256 digests of the reference's CSR (networkx
    neighbour order, vocab ids), which the test checks its rebuilt CSR against."""
    import hashlib
    tmp = os.path.join(HERE, f'_edges_{scale}_{n_edges}_{graph_seed}.npy')
    code = (f"import sys; sys.path.insert(0, {os.path.join(REPO, 'deepwalk-and-node2vec_amd')!r});"
            f"import numpy as np; from shallow_encoders.graph.rmat import rmat_edges;"
            f"e, _ = rmat_edges({scale}, {n_edges}, {graph_seed}); np.save({tmp!r}, e)")
    subprocess.run([sys.executable, '-c', code], check=True,
                   env=dict(os.environ, PYTHONDONTWRITEBYTECODE='1'))
    edges = np.load(tmp)
    os.remove(tmp)
    n = 1 << scale
    width = max(7, len(str(n)))
    g = nx.Graph()
    g.add_edges_from((f'n{u:0{width}d}', f'n{v:0{width}d}') for u, v in edges.tolist())
    del edges
    itos, stoi = vocab_of(g)
    assert len(itos) == n + 1
    row_ptr, col, _, _ = csr_of(g, stoi)
    deg = np.diff(row_ptr)
    hubs = np.argsort(-deg, kind='stable')[:n_hubs].astype(np.int32)
    starts = np.repeat(hubs, walks_per_hub)
    params = {'p': p, 'q': q} if method == 'node2vec' else None
    walker = ref_rwg.random_walk_factory(method, g, walk_length, params)
    random.seed(seed)
    walks = []
    with Capture() as cap:
        for s in starts:
            walks.append([stoi[t.lower()] for t in walker.walk(itos[s]).split()])
    walks = np.array(walks, dtype=np.int32)
    u = np.array(cap.uniforms, dtype=np.float64).reshape(len(starts), walk_length - 1)
    # the degree of the node each step was taken FROM (the row the pick was made in)
    step_deg = deg[walks[:, :-1]]
    print(f'{name}: hub degrees {deg[hubs].tolist()}; steps at rows of degree >= 10K: '
          f'{int((step_deg >= 10_000).sum())} of {step_deg.size}')
    save(name, scale=scale, n_edges=n_edges, graph_seed=graph_seed, seed=seed,
         walk_length=walk_length, method=np.array(method), p=p, q=q, starts=starts, uniforms=u,
         walks=walks, hub_degrees=deg[hubs],
         row_ptr_sha256=np.array(hashlib.sha256(row_ptr.astype('<i8').tobytes()).hexdigest()),
         col_sha256=np.array(hashlib.sha256(col.astype('<i4').tobytes()).hexdigest()))


def hub_fixtures():
    for scale, n_edges, tag in ((16, 600_000, 'rmat16'), (20, 10_000_000, 'rmat20')):
        hub_fixture(f'walks_{tag}_hubs_deepwalk.npz', scale, n_edges, 0, seed=61,
                    method='deepwalk', walk_length=10)
        hub_fixture(f'walks_{tag}_hubs_node2vec_p0.25_q4.npz', scale, n_edges, 0, seed=62,
                    method='node2vec', p=0.25, q=4.0)
        hub_fixture(f'walks_{tag}_hubs_node2vec_p1_q1.npz', scale, n_edges, 0, seed=63,
                    method='node2vec', p=1.0, q=1.0)


# ------------------------------------------------------------------------------- SGNS
def sg_windows(walks, R):
    """torch_dataset.py:300-309 (sg): centre text[i:i+1], targets text[i-R:i] | text[i+1:i+1+R]."""
    ins, tgts = [], []
    for text in walks:
        for i in range(R, len(text) - R):
            ins.append(text[i:i + 1])
            tgts.append(np.concatenate([text[i - R:i], text[i + 1:i + 1 + R]]))
    return np.stack(ins).astype(np.int64), np.stack(tgts).astype(np.int64)


def cbow_windows(walks, R):
    """torch_dataset.py:311-315 (cbow): inputs text[i-R:i] | text[i+1:i+1+R], target text[i]."""
    ins, tgts = sg_windows(walks, R)
    return tgts, ins


def reference_step(model, loss_fn, inputs, targets, noise):
    """trainer.py:131-152 wiring around the reference's own SkipGram / loss."""
    inputs_t = torch.as_tensor(inputs)
    outputs_t = torch.as_tensor(targets)
    nz = torch.as_tensor(noise).view(outputs_t.shape[0], -1)
    pos = model(inputs_t, outputs_t, proba=False)
    neg = model(inputs_t, nz, proba=False).view(outputs_t.shape[0], outputs_t.shape[1], -1)
    loss = loss_fn(pos, neg)
    recall = float((torch.sigmoid(pos) >= 0.5).float().mean())
    precision = float(1 - (torch.sigmoid(neg) >= 0.5).float().mean())
    return loss, recall, precision


def sgns_fixture(name, walks, V, d, R, K, lr, init_seed, noise_seed, n_steps=5, scale=1.0,
                 model_cls=None, mode='sg', max_norm=None):
    """F6: grads of one step, then params after 1 and n_steps Adam steps (new noise per step).
    model_cls / mode / max_norm: CBOW (model.py:94-110) with 'cbow' windows, and
    nn.Embedding(max_norm) renormalisation inside the reference's forwards."""
    torch.manual_seed(init_seed)
    model = (model_cls or SkipGram)(vocab_size=V, embedding_size=d, max_norm=max_norm)
    if scale != 1.0:
        with torch.no_grad():
            model._input_embedding.weight.mul_(scale)
            model._output_embedding.weight.mul_(scale)
    w_in0 = model._input_embedding.weight.detach().numpy().copy()
    w_out0 = model._output_embedding.weight.detach().numpy().copy()
    inputs, targets = (cbow_windows if mode == 'cbow' else sg_windows)(walks, R)
    B, C = targets.shape
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    renormed = None
    loss_fn = NegativeSamplingLoss()
    torch.manual_seed(noise_seed)
    noises, losses, recalls, precisions = [], [], [], []
    g_in = g_out = None
    p1 = None
    for step in range(n_steps):
        noise = generate_noise_batch(B, C, K, V).numpy()
        noises.append(noise)
        opt.zero_grad()
        loss, rec, prec = reference_step(model, loss_fn, inputs, targets, noise)
        loss['loss'].backward()
        if step == 0:
            g_in = model._input_embedding.weight.grad.numpy().copy()
            g_out = model._output_embedding.weight.grad.numpy().copy()
            renormed = (model._input_embedding.weight.detach().numpy().copy(),
                        model._output_embedding.weight.detach().numpy().copy())
        losses.append([float(loss['loss']), float(loss['positive-loss']),
                       float(loss['negative-loss'])])
        recalls.append(rec)
        precisions.append(prec)
        opt.step()
        if step == 0:
            p1 = (model._input_embedding.weight.detach().numpy().copy(),
                  model._output_embedding.weight.detach().numpy().copy())
    save(name, V=V, d=d, R=R, K=K, lr=lr, walks=np.asarray(walks, dtype=np.int32),
         inputs=inputs, targets=targets, noise=np.stack(noises), w_in0=w_in0, w_out0=w_out0,
         g_in=g_in, g_out=g_out, w_in1=p1[0], w_out1=p1[1],
         w_in_n=model._input_embedding.weight.detach().numpy(),
         w_out_n=model._output_embedding.weight.detach().numpy(),
         w_in0r=renormed[0], w_out0r=renormed[1], mode=mode,
         max_norm=np.nan if max_norm is None else max_norm,
         losses=np.array(losses), recall=np.array(recalls), precision=np.array(precisions))


def trajectory_fixture(name, seed, walks_per_node, walk_length, d, R, K, lr, batch_walks,
                       epochs, step_size, gamma):
    """F7: karate node2vec training for several epochs, StepLR per epoch (PL default)."""
    random.seed(seed)
    torch.manual_seed(seed)
    ds = ref_ds.KarateClubDataset(walks_per_node=walks_per_node, walk_length=walk_length,
                                  method='node2vec', method_params={'p': 1, 'q': 0.5})
    itos, stoi = vocab_of(ds.graph)
    V = len(itos)
    model = SkipGram(vocab_size=V, embedding_size=d, max_norm=None)
    w_in0 = model._input_embedding.weight.detach().numpy().copy()
    w_out0 = model._output_embedding.weight.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=step_size, gamma=gamma)
    loss_fn = NegativeSamplingLoss()
    all_walks, all_noise, losses, lrs, epoch_of_step = [], [], [], [], []
    for epoch in range(epochs):
        walks = [[stoi[t.lower()] for t in s.split()] for s in ds]
        for b0 in range(0, len(walks), batch_walks):
            batch = walks[b0:b0 + batch_walks]
            inputs, targets = sg_windows(batch, R)
            B, C = targets.shape
            noise = generate_noise_batch(B, C, K, V).numpy()
            opt.zero_grad()
            loss, _, _ = reference_step(model, loss_fn, inputs, targets, noise)
            loss['loss'].backward()
            opt.step()
            all_walks.append(np.asarray(batch, dtype=np.int32))
            all_noise.append(noise)
            losses.append(float(loss['loss']))
            lrs.append(opt.param_groups[0]['lr'])
            epoch_of_step.append(epoch)
        sched.step()
    save(name, seed=seed, V=V, d=d, R=R, K=K, lr=lr, step_size=step_size, gamma=gamma,
         epochs=epochs, walks=np.concatenate(all_walks), noise=np.concatenate(all_noise),
         batch_sizes=np.array([len(w) for w in all_walks]), w_in0=w_in0,
         w_out0=w_out0, losses=np.array(losses), lrs=np.array(lrs),
         epoch_of_step=np.array(epoch_of_step),
         w_in=model._input_embedding.weight.detach().numpy(),
         w_out=model._output_embedding.weight.detach().numpy())


SPLIT_CASES = [  # (class name, kwargs) of the reference's split algorithms
    ('TrainTestRatioSplit', {'train_ratio': 0.5}),
    ('TrainTestRatioSplit', {'train_ratio': 0.7, 'stratify': True}),
    ('TrainTestRatioSplit', {'train_ratio': 0.5, 'test_all': True}),
    ('TrainValTestRatioSplit', {'train_ratio': 0.6, 'val_ratio': 0.8}),
    ('TrainValTestRatioSplit', {'train_ratio': 0.5, 'val_ratio': 0.7, 'stratify': True}),
    ('TrainValTestStratifiedNSamplesSplit', {'train_samples': 3, 'val_samples': 2,
                                             'test_samples': 4}),
    ('TrainValTestStratifiedNSamplesSplit', {'train_samples': 3, 'val_samples': 2}),
]
SPLIT_SEEDS = (0, 7, 42)


def downstream_fixture(name):
    """Outputs of the reference's split algorithms (shallow_encoders/split/core.py) and edge
    operators (shallow_encoders/graph/edge_operators.py) on fixed inputs."""
    import shallow_encoders.split as ref_split
    from shallow_encoders.graph import edge_operators as ref_ops
    X = np.arange(40 * 3, dtype=np.float64).reshape(40, 3)
    y = np.asarray([0] * 14 + [1] * 13 + [2] * 13, dtype=np.float32)
    y = y[np.random.default_rng(3).permutation(40)]
    arrays = {'X': X, 'y': y}
    for i, (cls, kw) in enumerate(SPLIT_CASES):
        for seed in SPLIT_SEEDS:
            algo = getattr(ref_split, cls)(**kw)
            algo.random_state = seed
            for k, v in algo(X, y).items():
                arrays[f'split{i}_seed{seed}_{k}'] = v
    rng = np.random.default_rng(9)
    a, b = rng.normal(size=(6, 5)), rng.normal(size=(6, 5))
    arrays['op_lhs'], arrays['op_rhs'] = a, b
    for op in ('average', 'hadamard', 'weighted_l1', 'weighted_l2'):
        arrays[f'op_{op}'] = np.stack([ref_ops.edge_operator_factory(op)(a[j], b[j])
                                       for j in range(6)])
    save(name, **arrays)


def cbow_fixtures():
    """§8f 4: CBOW steps and max_norm renormalisation (reference model.py + nn.Embedding)."""
    from shallow_encoders.word2vec.model import CBOW
    rng = np.random.default_rng(41)
    sgns_fixture('sgns_cbow_d16_k3.npz', rng.integers(1, 40, size=(12, 9)), V=40, d=16, R=2,
                 K=3, lr=0.05, init_seed=8, noise_seed=9, model_cls=CBOW, mode='cbow')
    sgns_fixture('sgns_sg_maxnorm_d8_k2.npz', rng.integers(1, 30, size=(10, 8)), V=30, d=8, R=2,
                 K=2, lr=0.1, init_seed=10, noise_seed=11, scale=8.0, max_norm=1.0)
    sgns_fixture('sgns_cbow_maxnorm_d2_k1.npz', rng.integers(1, 6, size=(9, 8)), V=6, d=2, R=1,
                 K=1, lr=0.1, init_seed=12, noise_seed=13, scale=3.0, model_cls=CBOW,
                 mode='cbow', max_norm=1.0)


def trajectory128_fixture(name='traj_d128_k5_r5.npz', V=1025, d=128, R=5, K=5, lr=0.01, L=40,
                         batch_walks=16, steps=24, init_seed=51, noise_seed=52, walk_seed=53):
    """§8c trajectory parity at the bench's shape: >= 20 reference Adam steps at d=128, K=5,
    R=5, lr 0.01 (bench.py's lr) through the reference's SkipGram / NegativeSamplingLoss /
    generate_noise_batch + torch.optim.Adam (trainer.py:131-152 wiring). Walks are uniform ids
    (the SGNS step does not depend on where they come from); every step trains a new batch."""
    torch.manual_seed(init_seed)
    model = SkipGram(vocab_size=V, embedding_size=d, max_norm=None)
    w_in0 = model._input_embedding.weight.detach().numpy().copy()
    w_out0 = model._output_embedding.weight.detach().numpy().copy()
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    loss_fn = NegativeSamplingLoss()
    walks = np.random.default_rng(walk_seed).integers(1, V, size=(steps, batch_walks, L))
    torch.manual_seed(noise_seed)
    noises, losses = [], []
    for step in range(steps):
        inputs, targets = sg_windows(walks[step], R)
        B, C = targets.shape
        noise = generate_noise_batch(B, C, K, V).numpy()
        opt.zero_grad()
        loss, _, _ = reference_step(model, loss_fn, inputs, targets, noise)
        loss['loss'].backward()
        opt.step()
        noises.append(noise)
        losses.append([float(loss['loss']), float(loss['positive-loss']),
                       float(loss['negative-loss'])])
    save(name, V=V, d=d, R=R, K=K, lr=lr, init_seed=init_seed, noise_seed=noise_seed,
         walks=walks.astype(np.int16), noise=np.stack(noises).astype(np.int16), w_in0=w_in0,
         w_out0=w_out0, w_in=model._input_embedding.weight.detach().numpy(),
         w_out=model._output_embedding.weight.detach().numpy(), losses=np.array(losses))


CORA_SUBJECTS = ['Case_Based', 'Genetic_Algorithms', 'Neural_Networks',
                 'Probabilistic_Methods', 'Reinforcement_Learning', 'Rule_Learning', 'Theory']


def synthetic_cora(n_papers=240, n_cites=520, seed=17):
    """cora.cites / cora.content in the real files' format (tab-separated; content rows: paper
    id, 1,433 binary word features, subject). Paper ids are sparse ints as in Cora; citations
    include reverse duplicates (nx merges them) and every paper has at least one citation."""
    rng = np.random.default_rng(seed)
    ids = np.sort(rng.choice(np.arange(30, 1_200_000), size=n_papers, replace=False))
    pairs = [(int(ids[i]), int(ids[rng.integers(n_papers)])) for i in range(n_papers)]
    while len(pairs) < n_cites:
        a, b = rng.integers(n_papers, size=2)
        pairs.append((int(ids[a]), int(ids[b])))
    pairs += [(b, a) for a, b in pairs[:12]]          # reverse duplicates
    pairs = [(a, b) for a, b in pairs if a != b]
    cites = ''.join(f'{a}\t{b}\n' for a, b in pairs)
    rows = []
    for pid in rng.permutation(ids):
        feats = (rng.random(1433) < 0.013).astype(int)
        rows.append('\t'.join([str(pid)] + [str(x) for x in feats]
                              + [CORA_SUBJECTS[rng.integers(len(CORA_SUBJECTS))]]))
    return cites, ''.join(r + '\n' for r in rows)


def cora_fixture(name='walks_cora_node2vec_p1_q2.npz'):
    """§8 C2's ingest path: the reference's CoraDataset (datasets.py:183-221) on synthetic
    cora.cites / cora.content (the real files are not shipped), read through a temporary
    ASSETS_PATH: one epoch of node2vec p=1 q=2 walks (configs/sge_sg_cora.yaml's walker),
    the start order, the labels and a sample of the features."""
    import tempfile
    cites, content = synthetic_cora()
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, 'cora'))
        with open(os.path.join(tmp, 'cora', 'cora.cites'), 'w') as f:
            f.write(cites)
        with open(os.path.join(tmp, 'cora', 'cora.content'), 'w') as f:
            f.write(content)
        ref_ds.ASSETS_PATH = tmp

        def extra(ds):
            names = sorted(ds.labels)
            feat = np.stack([ds.features[n] for n in names[:16]]).astype(np.uint8)
            return dict(cites_txt=np.frombuffer(cites.encode(), np.uint8),
                        content_txt=np.frombuffer(content.encode(), np.uint8),
                        label_names=np.array(names), label_values=np.array(
                            [ds.labels[n] for n in names]),
                        feature_sample=feat, n_nodes=ds.graph.number_of_nodes(),
                        n_edges=ds.graph.number_of_edges())
        dataset_fixture(name, ref_ds.CoraDataset, seed=43, walks_per_node=2, walk_length=10,
                        method='node2vec', method_params={'p': 1, 'q': 2}, extra=extra)


def main():
    if sys.argv[1:] == ['cora']:
        cora_fixture()
        return
    if sys.argv[1:] == ['hubs']:
        hub_fixtures()
        return
    if sys.argv[1:] == ['traj128']:
        trajectory128_fixture()
        return
    if sys.argv[1:] == ['downstream']:
        downstream_fixture('downstream_split_ops.npz')
        return
    if sys.argv[1:] == ['cbow']:
        cbow_fixtures()
        return
    info = {'python': sys.version, 'torch': torch.__version__, 'networkx': nx.__version__}
    # F1/F4 karate node2vec (configs/sge_sg_karate_club.yaml walker) and a strongly biased p,q
    dataset_fixture('walks_karate_node2vec_p1_q0.5.npz', ref_ds.KarateClubDataset, seed=11,
                    walks_per_node=4, walk_length=10, method='node2vec',
                    method_params={'p': 1, 'q': 0.5})
    dataset_fixture('walks_karate_node2vec_p0.3_q3.npz', ref_ds.KarateClubDataset, seed=12,
                    walks_per_node=4, walk_length=12, method='node2vec',
                    method_params={'p': 0.3, 'q': 3})
    dataset_fixture('walks_karate_deepwalk.npz', ref_ds.KarateClubDataset, seed=13,
                    walks_per_node=4, walk_length=10, method='deepwalk')
    # F2 triplets (configs/sge_sg_graph_triplets.yaml walker)
    dataset_fixture('walks_triplets_deepwalk.npz', ref_ds.GraphTriplets, seed=14,
                    walks_per_node=8, walk_length=5, method='deepwalk')
    # F3 R-MAT scale 12 (4,096 nodes, power-law hubs), unweighted
    rmat_fixture('walks_rmat12_deepwalk.npz', 12, 40_000, 0, seed=21, n_walks=256,
                 walk_length=40, method='deepwalk')
    rmat_fixture('walks_rmat12_node2vec_p0.25_q4.npz', 12, 40_000, 0, seed=22, n_walks=96,
                 walk_length=30, method='node2vec', p=0.25, q=4.0)
    # F6 SGNS steps
    kz = np.load(os.path.join(HERE, 'walks_karate_node2vec_p1_q0.5.npz'))
    sgns_fixture('sgns_karate_d2_k1.npz', kz['walks'][:64], V=35, d=2, R=2, K=1, lr=0.1,
                 init_seed=0, noise_seed=1)
    rng = np.random.default_rng(5)
    sgns_fixture('sgns_d128_k5.npz', rng.integers(1, 256, size=(64, 10)), V=256, d=128, R=2, K=5,
                 lr=0.1, init_seed=2, noise_seed=3)
    sgns_fixture('sgns_d256_k5_r5.npz', rng.integers(0, 128, size=(8, 16)), V=128, d=256, R=5,
                 K=5, lr=0.05, init_seed=4, noise_seed=5)
    sgns_fixture('sgns_clamp_d8_k2.npz', rng.integers(1, 64, size=(32, 9)), V=64, d=8, R=2, K=2,
                 lr=0.1, init_seed=6, noise_seed=7, scale=40.0)
    # F7 trajectory with StepLR
    trajectory_fixture('traj_karate_node2vec.npz', seed=31, walks_per_node=8, walk_length=10,
                       d=2, R=2, K=1, lr=0.1, batch_walks=64, epochs=3, step_size=1, gamma=0.5)
    # §8f 3: downstream split algorithms + edge operators
    downstream_fixture('downstream_split_ops.npz')
    cbow_fixtures()
    cora_fixture()
    trajectory128_fixture()
    with open(os.path.join(HERE, 'golden_info.json'), 'w') as f:
        json.dump(info, f, indent=2)


if __name__ == '__main__':
    main()
