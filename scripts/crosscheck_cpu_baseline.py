"""Cross-check of the CPU baseline port against the reference itself (BASELINE.md:63).

    PYTHONDONTWRITEBYTECODE=1 python scripts/crosscheck_cpu_baseline.py > profiles/r02_cpu_crosscheck.log

Runs in the build container only (the reference never travels to the GPU box). On the same
inputs, times the reference's own code and the oracle port bench.py's cpu_baseline uses, and
checks that their outputs are identical:
  * walkers on the C3 graph (R-MAT 20, the product's edge list, as a networkx graph with
    n%07d names): the reference's DeepWalk / Node2Vec (random_walk_generator.py:61-119) under a
    captured `random` stream vs oracle/walk_ref.py's deepwalk_walk / node2vec_walk(listscan)
    replaying those uniforms, 1 core;
  * the SGNS step at V = 1,048,577, d = 128, K = 5, R = 5: the reference's SkipGram
    (model.py:79-91) + NegativeSamplingLoss (loss.py:14-22) + torch.optim.Adam wired as
    trainer.py:131-152 vs oracle/sgns_ref.TorchAdamRef, at 64 / 1,024 / 8,192 walks per step.
Prints one JSON line per comparison and a summary line.
"""
import json
import os
import random
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.dont_write_bytecode = True
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))
sys.path.insert(0, REPO)

import make_golden as mg  # noqa: E402  (imports the reference's shallow_encoders)
from oracle import sgns_ref, walk_ref  # noqa: E402

THREADS = int(os.environ.get('CROSSCHECK_THREADS', '8'))


class Uniforms:
    """Records the doubles the reference's random.choices consumes (random._inst.random); unlike
    make_golden.Capture it does not copy every choices() population, so the reference is timed
    at its own speed."""

    def __enter__(self):
        self.values = []
        orig = self._orig = random._inst.random
        rec = self.values.append

        def wrapped():
            u = orig()
            rec(u)
            return u
        random._inst.random = wrapped
        return self

    def __exit__(self, *exc):
        del random._inst.random
        return False


def emit(**kw):
    print(json.dumps(kw), flush=True)


def rmat20_graph():
    import subprocess
    import networkx as nx
    tmp = os.path.join('/tmp', 'crosscheck_edges.npy')
    code = (f"import sys; sys.path.insert(0, {os.path.join(REPO, 'deepwalk-and-node2vec_amd')!r});"
            f"import numpy as np; from shallow_encoders.graph.rmat import rmat_edges;"
            f"e, _ = rmat_edges(20, 10_000_000, 0); np.save({tmp!r}, e)")
    subprocess.run([sys.executable, '-c', code], check=True,
                   env=dict(os.environ, PYTHONDONTWRITEBYTECODE='1'))
    edges = np.load(tmp)
    os.remove(tmp)
    g = nx.Graph()
    g.add_edges_from((f'n{u:07d}', f'n{v:07d}') for u, v in edges.tolist())
    itos, stoi = mg.vocab_of(g)
    row_ptr, col, _, _ = mg.csr_of(g, stoi)
    t0 = time.perf_counter()
    port_graph = walk_ref.NxLikeGraph(row_ptr, col, itos)
    print(f'# port graph (oracle NxLikeGraph from the CSR) built in {time.perf_counter() - t0:.1f}s',
          flush=True)
    return g, itos, stoi, port_graph


def walkers(budget_s=20.0):
    g, itos, stoi, csr = rmat20_graph()
    n = len(itos) - 1
    rng = np.random.default_rng(0)
    for method, L, params in (('deepwalk', 80, None), ('node2vec', 10, {'p': 1.0, 'q': 1.0}),
                              ('node2vec', 10, {'p': 0.25, 'q': 4.0})):
        walker = mg.ref_rwg.random_walk_factory(method, g, L, params)
        random.seed(1)
        starts, walks = [], []
        with Uniforms() as cap:
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < budget_s:
                s = int(rng.integers(1, n + 1))
                starts.append(s)
                walks.append(walker.walk(itos[s]).split())
            t_ref = time.perf_counter() - t0
        u = np.array(cap.values).reshape(len(starts), L - 1)
        t0 = time.perf_counter()
        port = []
        for s, uu in zip(starts, u):
            if method == 'deepwalk':
                port.append(walk_ref.deepwalk_walk(csr, itos[s], L, uu.tolist()))
            else:
                port.append(walk_ref.node2vec_walk(csr, itos[s], L, params['p'], params['q'],
                                                   uu.tolist(), listscan=True))
        t_port = time.perf_counter() - t0
        steps = len(starts) * (L - 1)
        emit(kind='walker', method=method, params=params, walk_length=L, walks=len(starts),
             identical=port == walks, ref_steps_per_s=steps / t_ref,
             port_steps_per_s=steps / t_port, port_over_ref=t_ref / t_port, cores=1)
    del g


def sgns(batches=(64, 1024, 8192)):
    torch.set_num_threads(THREADS)
    V, d, R, K, L, lr = 1_048_577, 128, 5, 5, 80, 0.01
    loss_fn = mg.NegativeSamplingLoss()
    rng = np.random.default_rng(0)
    for bw in batches:
        torch.manual_seed(0)
        model = mg.SkipGram(vocab_size=V, embedding_size=d, max_norm=None)
        w_in0 = model._input_embedding.weight.detach().numpy().copy()
        w_out0 = model._output_embedding.weight.detach().numpy().copy()
        opt = torch.optim.Adam(model.parameters(), lr=lr)
        port = sgns_ref.TorchAdamRef(w_in0, w_out0, lr=lr)
        n_steps = 3 if bw <= 1024 else 2
        t_ref = t_port = 0.0
        same_loss = True
        pairs = 0
        for step in range(n_steps):
            walks = rng.integers(1, V, size=(bw, L))
            ins, tgt = sgns_ref.sg_windows(walks, R)
            noise = rng.integers(0, V, size=(len(ins), 2 * R, K))
            t0 = time.perf_counter()
            opt.zero_grad()
            loss, _, _ = mg.reference_step(model, loss_fn, ins, tgt, noise)
            loss['loss'].backward()
            opt.step()
            dt_ref = time.perf_counter() - t0
            t0 = time.perf_counter()
            pl = port.train_step(ins, tgt, noise)
            dt_port = time.perf_counter() - t0
            same_loss &= float(loss['loss']) == pl['loss']
            if step > 0:                        # step 0 allocates the Adam state
                t_ref += dt_ref
                t_port += dt_port
                pairs += tgt.size
        w_in, w_out = port.tables()
        identical = (same_loss and np.array_equal(w_in, model._input_embedding.weight.detach().numpy())
                     and np.array_equal(w_out, model._output_embedding.weight.detach().numpy()))
        emit(kind='sgns', batch_walks=bw, timed_steps=n_steps - 1, identical=bool(identical),
             ref_pairs_per_s=pairs / t_ref, port_pairs_per_s=pairs / t_port,
             port_over_ref=t_ref / t_port, threads=THREADS)
        del model, opt, port


def main():
    print(f'# host: {os.cpu_count()} CPUs; python {sys.version.split()[0]}; torch '
          f'{torch.__version__}; reference imported from {os.path.dirname(mg.ref_rwg.__file__)}',
          flush=True)
    what = sys.argv[1:] or ['walkers', 'sgns']
    if 'walkers' in what:
        walkers()
    if 'sgns' in what:
        sgns()


if __name__ == '__main__':
    main()
