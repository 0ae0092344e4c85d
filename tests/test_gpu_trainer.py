"""End-to-end training on the MI355X: the reference's trajectory (loss curve + final tables,
StepLR) through Word2VecTrainer + HIP Adam, and the tools/train.py CLI.

Tolerances: per-step loss rtol 1e-4, final tables rtol 1e-4 / atol 1e-5 (fp32, atomic
accumulation order differs from torch's embedding backward)."""
import os
import random

import numpy as np
import pytest
import torch

from conftest import golden

from shallow_encoders.word2vec.dataloader.torch_dataset import W2VCollateFunctional
from shallow_encoders.word2vec.model import SkipGram
from shallow_encoders.word2vec.optim import Adam
from shallow_encoders.word2vec.trainer import Word2VecTrainer

pytestmark = pytest.mark.gpu


def _reference_run(f, manual_grads=True):
    torch.manual_seed(int(f['seed']))
    # the fixture drew the node2vec walks with `random` and the model + noise with torch's
    # global generator (model init first); the walks are replayed from the fixture here
    V, d = int(f['V']), int(f['d'])
    model = SkipGram(V, d)
    np.testing.assert_array_equal(model.input_embedding.numpy(), f['w_in0'])
    model = model.cuda()
    opt = Adam(model.parameters(), lr=float(f['lr']))
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=int(f['step_size']),
                                            gamma=float(f['gamma']))
    tr = Word2VecTrainer(model, opt, sched, neg_samples=int(f['K']), vocab_size=V, noise='torch')
    tr.manual_grads = manual_grads
    collate = W2VCollateFunctional('sg', int(f['R']), 256)
    offs = np.concatenate([[0], np.cumsum(f['batch_sizes'])])
    losses, epoch = [], 0
    for step in range(len(f['batch_sizes'])):
        if f['epoch_of_step'][step] != epoch:
            sched.step()
            epoch = int(f['epoch_of_step'][step])
        walks = torch.as_tensor(f['walks'][offs[step]:offs[step + 1]]).long()
        batch = collate(list(walks))
        out = tr.training_step(batch)
        if not manual_grads:
            out['loss'].backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(out['loss'].detach()))
    return model, losses


@pytest.mark.parametrize('manual_grads', [True, False])
def test_trajectory_matches_reference(manual_grads, hip_device):
    f = golden('traj_karate_node2vec.npz')
    model, losses = _reference_run(f, manual_grads)
    np.testing.assert_allclose(losses, f['losses'], rtol=1e-4)
    from oracle import sgns_ref
    from test_gpu_sgns import assert_within_envelope, reference_envelope
    offs = np.concatenate([[0], np.cumsum(f['batch_sizes'])])
    batches, noff = [], 0
    for step in range(len(f['batch_sizes'])):
        ins, tgt = sgns_ref.sg_windows(f['walks'][offs[step]:offs[step + 1]], int(f['R']))
        batches.append((ins, tgt, f['noise'][noff:noff + len(ins)], float(f['lrs'][step])))
        noff += len(ins)
    ex_in, ex_out = reference_envelope(f['w_in0'], f['w_out0'], float(f['lr']), batches)
    lr = float(f['lr'])
    assert_within_envelope(model.input_embedding.numpy(), f['w_in'], ex_in, lr, rtol=1e-4,
                           atol=1e-5)
    assert_within_envelope(model.output_embedding.numpy(), f['w_out'], ex_out, lr, rtol=1e-4,
                           atol=1e-5)


def test_train_cli_karate_end_to_end(tmp_path, hip_device):
    from tools import train as train_tool
    out = str(tmp_path / 'runs')
    overrides = [f'path.output_dir={out}', f'output_dir={out}', 'train.max_epochs=4',
                 'datamodule.additional_parameters.walks_per_node=16',
                 'datamodule.additional_parameters.rng=philox', 'train.noise=device']
    last = train_tool.main(['--config-name', 'sge_sg_karate_club'] + overrides)
    assert last['train-epoch/loss'] == last['train-epoch/loss']
    ck = os.path.join(out, 'graph_karate_club', 'SG_exp01_baseline', 'checkpoints')
    files = sorted(os.listdir(ck))
    assert 'last.ckpt' in files and len(files) == 5
    assert files[0] == 'checkpoint_epoch=000000_step=000000009.ckpt'
    state = torch.load(os.path.join(ck, 'last.ckpt'), weights_only=True)
    assert set(state['state_dict']) == {'_model._input_embedding.weight',
                                        '_model._output_embedding.weight'}
    # reload for analysis like tools/model_analysis.py does
    from shallow_encoders.config_parser import load_config
    cfg = load_config('sge_sg_karate_club', overrides=overrides[2:])
    ds = cfg.datamodule.instantiate_dataset()
    tr = cfg.instantiate_trainer(dataset=ds, checkpoint_path=os.path.join(ck, 'last.ckpt'))
    np.testing.assert_array_equal(tr.model.input_embedding.numpy(),
                                  state['state_dict']['_model._input_embedding.weight'].numpy())
    hist = os.path.join(out, 'graph_karate_club', 'SG_exp01_baseline', 'run_history')
    assert len(os.listdir(hist)) == 1


def test_training_reduces_loss_on_triplets(tmp_path, hip_device):
    from tools import train as train_tool
    out = str(tmp_path / 'runs')
    first = train_tool.main(['--config-name', 'sge_sg_graph_triplets', f'path.output_dir={out}',
                             f'output_dir={out}', 'train.max_epochs=1'])
    more = train_tool.main(['--config-name', 'sge_sg_graph_triplets', f'path.output_dir={out}',
                            f'output_dir={out}', 'train.max_epochs=5'])
    assert more['train-epoch/loss'] < first['train-epoch/loss'] + 0.05


def test_downstream_quality_karate(tmp_path, hip_device):
    """Train karate with the reference config (node2vec p=1 q=0.5, d=2, 50 epochs) and run the
    downstream tool: README.md:276-281 reports 98.06% node / 69.52% edge accuracy (means over
    100 / 1000 experiments) for the reference's own training."""
    from tools import graph_model_downstream_classification as downstream
    from tools import train as train_tool
    out = str(tmp_path / 'runs')
    base = [f'path.output_dir={out}', f'output_dir={out}']
    train_tool.main(['--config-name', 'sge_sg_karate_club'] + base)
    res = downstream.main(['--config-name', 'sge_sg_karate_club'] + base + [
        'downstream.node_classification.n_experiments=20',
        'downstream.edge_classification.n_experiments=100'])
    print(res)
    assert res['node_accuracy'] >= 0.93, res
    assert res['edge_accuracy'] >= 0.64, res
    assert os.path.exists(os.path.join(out, 'graph_karate_club', 'SG_exp01_baseline', 'analysis',
                                       'downstream-node-classification.jpg'))


@pytest.mark.parametrize('config,mode', [('w2v_cbow_abcde', 'cbow'), ('w2v_sg_abcde', 'sg')])
def test_text_word2vec_abcde(tmp_path, hip_device, config, mode):
    """Text word2vec through tools/train.py: the reference's abcde configs
    (max_norm 1.0, renormalised on every lookup; the per-step parity of that is in
    test_gpu_sgns.py) — CBOW over real (B, 2R) -> (B, 1) batches and skip-gram: the loss falls
    and co-occurring words score higher than words that never meet (README.md:127-147: `a`
    goes with `b`, `c` with `d`)."""
    from tools import train as train_tool
    out = str(tmp_path / 'runs')
    last = train_tool.main(['--config-name', config, f'path.output_dir={out}',
                            f'output_dir={out}', f'datamodule.mode={mode}',
                            'datamodule.num_workers=0', 'train.max_epochs=40'])
    assert last['train-epoch/loss'] < 1.3, last
    ck = os.path.join(out, 'abcde', 'CBOW_exp01_baseline' if 'cbow' in config
                      else 'SG_exp01_baseline', 'checkpoints', 'last.ckpt')
    sd = torch.load(ck, weights_only=True)['state_dict']
    w_in = sd['_model._input_embedding.weight'].numpy()
    w_out = sd['_model._output_embedding.weight'].numpy()
    from shallow_encoders.config_parser import load_config
    vocab = load_config(config).datamodule.instantiate_dataset().vocab
    i = {t: w_in[vocab[t]] for t in 'abcd'}
    o = {t: w_out[vocab[t]] for t in 'abcd'}
    assert np.dot(i['a'], o['b']) > np.dot(i['a'], o['c'])
    assert np.dot(i['c'], o['d']) > np.dot(i['c'], o['a'])


@pytest.mark.parametrize('d', [64, 128])
def test_fused_trainer_step_equals_unfused(hip_device, d):
    """Walk batches with the HIP Adam: training_step applies the update itself (output-table
    Adam fused into the records gather, input-table Adam overlapped on a side stream into a
    second buffer), and the tables, Adam state and losses equal SGNS + optimizer.step() (the
    unfused form, fuse_into_sgns=False) up to float-atomic summation order."""
    from shallow_encoders.graph.random_walk_generator import DeepWalk
    from shallow_encoders.graph.rmat import rmat_graph
    from test_gpu_sgns import assert_params_close
    csr = rmat_graph(12, 40_000, 0, device=hip_device)
    walker = DeepWalk(csr, 30, rng='philox', seed=3, device=hip_device)
    V, R, K, lr = csr.vocab_size, 3, 4, 0.02
    runs = []
    for fuse in (True, False):
        torch.manual_seed(11)
        model = SkipGram(V, d).cuda()
        opt = Adam(model.parameters(), lr=lr, fuse_into_sgns=fuse)
        sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1, gamma=0.5)
        tr = Word2VecTrainer(model, opt, sched, neg_samples=K, vocab_size=V, noise='device',
                             seed=5, context_radius=R)
        tr.manual_grads = True
        losses = []
        for step in range(5):
            if step == 3:
                sched.step()                       # lr change between steps
            starts = torch.randint(1, V, (300,), generator=torch.Generator().manual_seed(step),
                                   dtype=torch.int32).to(hip_device)
            out = tr.training_step(walker.walk_batch(starts, walk_id0=step * 300))
            opt.step()
            opt.zero_grad()
            losses.append(out['loss'])
        torch.cuda.synchronize()
        assert bool(opt._alt) == fuse               # the fused path ran (second buffer exists)
        assert float(model.input_weight.grad.abs().max()) == 0.0
        assert float(model.output_weight.grad.abs().max()) == 0.0
        runs.append((model, opt, [float(x) for x in losses]))
    (mf, of, lf), (mu, ou, lu) = runs
    np.testing.assert_allclose(lf, lu, rtol=1e-4)
    for a, b in ((mf.input_weight, mu.input_weight), (mf.output_weight, mu.output_weight)):
        assert_params_close(a.detach().cpu().numpy(), b.detach().cpu().numpy(), lr,
                            max_frac=5e-3, max_abs=2.05 * lr * 5)
    for pf, pu in zip(mf.parameters(), mu.parameters()):
        assert float(of.state[pf]['step']) == float(ou.state[pu]['step']) == 5.0
        np.testing.assert_allclose(of.state[pf]['exp_avg'].cpu().numpy(),
                                   ou.state[pu]['exp_avg'].cpu().numpy(), rtol=1e-3, atol=1e-6)


def test_d128_trajectory_matches_reference(hip_device):
    """24 reference training steps at the bench's shape (d=128, K=5, R=5, lr 0.01;
    traj_d128_k5_r5.npz from the reference's SkipGram / loss / generate_noise_batch +
    torch.optim.Adam) through the user-facing fused step: Word2VecTrainer.training_step on
    device walk batches with noise='torch' (the reference's negative stream) and the HIP Adam
    (out-table Adam fused into the records gather, in-table Adam on the side stream).

    Stated tolerance: per-step loss rtol 1e-4; final tables rtol 1e-4 / atol 1e-5 on at least
    99.99% of the entries and no entry off by more than lr / 10 (an entry whose gradient is a
    near-cancelling sum can have its Adam step flipped by the summation order). The envelope
    of the reference itself against its float64-exact-sum rerun is printed for comparison."""
    from oracle import sgns_ref
    f = golden('traj_d128_k5_r5.npz')
    V, d, R, K, lr = int(f['V']), int(f['d']), int(f['R']), int(f['K']), float(f['lr'])
    torch.manual_seed(int(f['init_seed']))
    model = SkipGram(V, d)
    np.testing.assert_array_equal(model.input_embedding.numpy(), f['w_in0'])
    np.testing.assert_array_equal(model.output_embedding.numpy(), f['w_out0'])
    model = model.cuda()
    opt = Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=1000, gamma=1.0)
    tr = Word2VecTrainer(model, opt, sched, neg_samples=K, vocab_size=V, noise='torch',
                         context_radius=R)
    tr.manual_grads = True
    torch.manual_seed(int(f['noise_seed']))
    losses = []
    for step in range(f['walks'].shape[0]):
        walks = torch.as_tensor(f['walks'][step].astype(np.int32)).to(hip_device)
        out = tr.training_step(walks)
        opt.step()
        opt.zero_grad()
        losses.append(float(out['loss']))
    assert bool(opt._alt)                         # the fused step ran
    np.testing.assert_allclose(losses, f['losses'][:, 0], rtol=1e-4)
    batches = []
    for step in range(f['walks'].shape[0]):
        ins, tgt = sgns_ref.sg_windows(f['walks'][step].astype(np.int64), R)
        batches.append((ins, tgt, f['noise'][step].astype(np.int64)))
    from test_gpu_sgns import reference_envelope
    ex_in, ex_out = reference_envelope(f['w_in0'], f['w_out0'], lr, batches)
    for name, got, exp, ex in (('w_in', model.input_embedding.numpy(), f['w_in'], ex_in),
                               ('w_out', model.output_embedding.numpy(), f['w_out'], ex_out)):
        bad = ~np.isclose(got, exp, rtol=1e-4, atol=1e-5)
        bad_ex = ~np.isclose(ex, exp, rtol=1e-4, atol=1e-5)
        print(f'{name}: {bad.sum()} / {bad.size} outside rtol 1e-4 / atol 1e-5, max |diff| '
              f'{np.abs(got - exp).max():.3e}; reference vs its exact-sum rerun: {bad_ex.sum()} '
              f'outside, max |diff| {np.abs(ex - exp).max():.3e}')
        assert bad.mean() <= 1e-4, f'{name}: {bad.sum()} entries outside tolerance'
        assert np.abs(got - exp).max() <= lr / 10


def _record_step_losses(monkeypatch):
    """Records the loss of every eager training_step (1 step) and of every graph replay (the
    mean over its n steps) as (n, loss) in call order."""
    rec = []
    orig_step = Word2VecTrainer.training_step
    orig_push = Word2VecTrainer.push_replayed

    def step(self, batch, *a, **k):
        out = orig_step(self, batch, *a, **k)
        if out is not None:   # (None: a step being captured into a graph)
            rec.append((1, out['loss'].detach().clone()))
        return out

    def push(self, terms, n):
        rec.append((n, terms['loss'].detach().clone()))
        return orig_push(self, terms, n)
    monkeypatch.setattr(Word2VecTrainer, 'training_step', step)
    monkeypatch.setattr(Word2VecTrainer, 'push_replayed', push)
    return rec


def _first_step_losses(rec, unroll: int = 16):
    """(loss of step 0, mean loss of steps 1..unroll) of the first epoch from a _record_step_losses
    record: an eager run logs them one by one, a graphed run as step 0 and one replay."""
    if rec[1][0] == unroll:
        return float(rec[0][1]), float(rec[1][1])
    assert all(n == 1 for n, _ in rec[:unroll + 1])
    return float(rec[0][1]), float(np.mean([float(x) for _, x in rec[1:unroll + 1]]))


# The float-mode loops hold the graphed runs to the eager run step by step over the first 17
# steps (step 0, then the first graph's 16), at the per-step bar: before float-atomic order
# differences compound through Adam's normalised steps. The whole loop is pinned bit for bit in
# the deterministic mode (test_gpu_exact.py::test_exact_train_loop_eager_twice_and_graphs_
# bit_identical, test_reference_streams_c2_loop_graphed_deterministic below).
FIRST_STEPS_RTOL = 1e-4


def test_train_loop_replays_graphs_equal_to_eager(tmp_path, hip_device, monkeypatch):
    """tools/train.py on the C2 shape (Cora-sized R-MAT, node2vec, L = 10, R = 2, 64-walk
    batches, d = 128) with Philox walks and device negatives: word2vec/fit.py replays the steps
    as HIP graphs of 16 (GraphedTrainerStep) after each epoch's first batch, and trains what the
    eager loop (DW_TRAIN_GRAPH=0) trains — the same number of steps, Adam step counts and walks
    (the dataset's epoch position), and the same losses over the first 17 steps at the per-step
    bar (below)."""
    from tools import train as train_tool
    from shallow_encoders.word2vec import graphed
    replays = []
    orig = graphed.GraphedTrainerStep.replay

    def counting(self):
        replays.append(self.unroll)
        return orig(self)
    monkeypatch.setattr(graphed.GraphedTrainerStep, 'replay', counting)
    rec = _record_step_losses(monkeypatch)
    lr = 0.01
    base = ['datamodule.dataset_name=graph_rmat', 'datamodule.additional_parameters.scale=12',
            'datamodule.additional_parameters.n_edges=5429',
            'datamodule.additional_parameters.graph_seed=0',
            'datamodule.additional_parameters.walks_per_node=1',
            'datamodule.additional_parameters.method_params.q=1',
            'datamodule.additional_parameters.rng=philox', 'train.noise=device',
            'model.embedding_size=128', f'train.optimizer.lr={lr}', 'train.max_epochs=2']
    runs, firsts = [], []
    for mode, scatter in (('0', 'auto'), ('1', 'records'), ('1', 'auto')):
        rec.clear()
        monkeypatch.setenv('DW_TRAIN_GRAPH', mode)
        monkeypatch.setenv('DW_TRAIN_GRAPH_SCATTER', scatter)
        out = str(tmp_path / f'runs{mode}{scatter}')
        torch.manual_seed(0)
        random.seed(0)   # the start-node shuffle (datasets.py:45,86-88: the global generator)
        last = train_tool.main(['--config-name', 'sge_sg_cora', f'path.output_dir={out}',
                                f'output_dir={out}', f'train.experiment=g{mode}'] + base)
        ck = os.path.join(out, 'graph_rmat', f'g{mode}', 'checkpoints', 'last.ckpt')
        state = torch.load(ck, weights_only=True)
        runs.append((last, state))
        firsts.append(_first_step_losses(rec))
    # 4,096 walks / 64 = 64 batches per epoch: 1 eager + 3 graphs of 16 + 15 eager, two epochs
    assert replays == [16] * 12
    (l0, s0), (l1, s1), (l2, s2) = runs
    assert s0['global_step'] == s1['global_step'] == s2['global_step'] == 128
    # In the float mode the loop is not bit-reproducible run to run, eager or graphed: float
    # atomics (the centre gradients, chunk-boundary rows) sum in a run-dependent order, and
    # Adam's normalised steps turn the resulting sign noise on g ~ 0 entries into lr-sized moves
    # that compound over 128 steps at lr = 0.01. So the graphs (records step, and the default
    # atomic scatter) are held to the eager loop at the per-step bar over the first 17 steps
    # (FIRST_STEPS_RTOL), with the same steps, walks, negatives and Adam step counts (above).
    # Each graphed step itself is checked against the eager step from the same state in
    # test_gpu_graphed.py, and in the deterministic mode the same loop's eager and graphed runs
    # end with bit-identical tables.
    for f in firsts[1:]:
        np.testing.assert_allclose(f, firsts[0], rtol=FIRST_STEPS_RTOL)


def _karate_fit(f, graph: str, monkeypatch):
    """The reference's karate node2vec trajectory (traj_karate_node2vec.npz: random.seed and
    torch.manual_seed(seed), the dataset, SkipGram, Adam + StepLR per epoch, 64-walk batches,
    noise from torch's generator) through word2vec/fit.py with the reference's own streams
    (rng='python' walks, noise='torch'); graph='1' replays the middle batches of every epoch as
    HIP graphs of 2 (GraphedTrainerStep: both streams generated in HBM)."""
    import random
    from shallow_encoders.config_parser.core import WalkBatchLoader
    from shallow_encoders.word2vec.dataloader.torch_dataset import GraphDataset
    from shallow_encoders.word2vec.fit import fit
    monkeypatch.setenv('DW_TRAIN_GRAPH', graph)
    seed = int(f['seed'])
    random.seed(seed)
    torch.manual_seed(seed)
    ds = GraphDataset('graph_karate_club', context_radius=int(f['R']),
                      additional_parameters={'walks_per_node': 8, 'walk_length': 10,
                                             'method': 'node2vec',
                                             'method_params': {'p': 1, 'q': 0.5}})
    V, d = int(f['V']), int(f['d'])
    model = SkipGram(V, d)
    np.testing.assert_array_equal(model.input_embedding.numpy(), f['w_in0'])
    model = model.cuda()
    opt = Adam(model.parameters(), lr=float(f['lr']))
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=int(f['step_size']),
                                            gamma=float(f['gamma']))
    tr = Word2VecTrainer(model, opt, sched, neg_samples=int(f['K']), vocab_size=V, noise='torch',
                         context_radius=int(f['R']))
    epochs = []
    orig = tr.on_train_epoch_end

    def epoch_end():
        out = orig()
        epochs.append(out)
        return out
    tr.on_train_epoch_end = epoch_end
    fit(tr, WalkBatchLoader(ds, 64), max_epochs=int(f['epochs']), verbose=False, graph_unroll=2)
    return model, epochs, random.getstate(), torch.get_rng_state()


def test_karate_trajectory_through_graphed_loop(hip_device, monkeypatch):
    """the reference's configs with their own streams on the graphed loop. The
    karate trajectory fixture (the reference's dataset, model, noise and StepLR) replayed through
    fit() with graphs of 2 steps: per-epoch mean losses at the fixture's bar (rtol 1e-4), final
    tables inside the reference's own envelope, and `random` / torch's generator left bit-equal
    to the eager loop's (so every walk and negative was the reference's)."""
    from shallow_encoders.word2vec import graphed
    replays = []
    orig = graphed.GraphedTrainerStep.replay

    def counting(self):
        replays.append((self.mt_walks is not None, self.mt_noise is not None))
        return orig(self)
    monkeypatch.setattr(graphed.GraphedTrainerStep, 'replay', counting)
    f = golden('traj_karate_node2vec.npz')
    model, epochs, py_state, t_state = _karate_fit(f, '1', monkeypatch)
    assert replays == [(True, True)] * int(f['epochs'])   # one graph of 2 per epoch
    eo = f['epoch_of_step']
    for e, got in enumerate(epochs):
        np.testing.assert_allclose(got['train-epoch/loss'], f['losses'][eo == e].mean(),
                                   rtol=1e-4)
    from oracle import sgns_ref
    from test_gpu_sgns import assert_within_envelope, reference_envelope
    offs = np.concatenate([[0], np.cumsum(f['batch_sizes'])])
    batches, noff = [], 0
    for step in range(len(f['batch_sizes'])):
        ins, tgt = sgns_ref.sg_windows(f['walks'][offs[step]:offs[step + 1]], int(f['R']))
        batches.append((ins, tgt, f['noise'][noff:noff + len(ins)], float(f['lrs'][step])))
        noff += len(ins)
    ex_in, ex_out = reference_envelope(f['w_in0'], f['w_out0'], float(f['lr']), batches)
    lr = float(f['lr'])
    assert_within_envelope(model.input_embedding.numpy(), f['w_in'], ex_in, lr, rtol=1e-4,
                           atol=1e-5)
    assert_within_envelope(model.output_embedding.numpy(), f['w_out'], ex_out, lr, rtol=1e-4,
                           atol=1e-5)
    _, eager_epochs, py_eager, t_eager = _karate_fit(f, '0', monkeypatch)
    assert py_state == py_eager
    assert torch.equal(t_state, t_eager)
    for a, b in zip(epochs, eager_epochs):
        np.testing.assert_allclose(a['train-epoch/loss'], b['train-epoch/loss'], rtol=1e-4)


def test_reference_streams_c2_loop_graphed(tmp_path, hip_device, monkeypatch):
    """tools/train.py --config-name=sge_sg_cora on the Cora-shaped R-MAT with the reference's
    own streams (rng: python walks, noise: torch) replays its steps as graphs of 16 and leaves
    `random` and torch's generator exactly where the eager loop leaves them (the same walks and
    negatives, step for step), with the same step count and epoch losses within the loop's
    per-step losses over the first 17 steps."""
    import random
    from tools import train as train_tool
    from shallow_encoders.word2vec import graphed
    replays = []
    orig = graphed.GraphedTrainerStep.replay

    def counting(self):
        replays.append(self.unroll)
        return orig(self)
    monkeypatch.setattr(graphed.GraphedTrainerStep, 'replay', counting)
    rec = _record_step_losses(monkeypatch)
    base = ['datamodule.dataset_name=graph_rmat', 'datamodule.additional_parameters.scale=12',
            'datamodule.additional_parameters.n_edges=5429',
            'datamodule.additional_parameters.graph_seed=0',
            'datamodule.additional_parameters.walks_per_node=1',
            'datamodule.additional_parameters.method_params.q=1',
            'datamodule.additional_parameters.rng=python', 'train.noise=torch',
            'model.embedding_size=128', 'train.optimizer.lr=0.01', 'train.max_epochs=2']
    runs, firsts = [], []
    for mode in ('0', '1'):
        rec.clear()
        monkeypatch.setenv('DW_TRAIN_GRAPH', mode)
        out = str(tmp_path / f'runs{mode}')
        random.seed(5)
        torch.manual_seed(0)
        last = train_tool.main(['--config-name', 'sge_sg_cora', f'path.output_dir={out}',
                                f'output_dir={out}', f'train.experiment=g{mode}'] + base)
        ck = os.path.join(out, 'graph_rmat', f'g{mode}', 'checkpoints', 'last.ckpt')
        state = torch.load(ck, weights_only=True)
        runs.append((last, state, random.getstate(), torch.get_rng_state()))
        firsts.append(_first_step_losses(rec))
    assert replays == [16] * 6
    (l0, s0, r0, t0), (l1, s1, r1, t1) = runs
    assert s0['global_step'] == s1['global_step'] == 128
    assert r0 == r1 and torch.equal(t0, t1)
    np.testing.assert_allclose(firsts[1], firsts[0], rtol=FIRST_STEPS_RTOL)


def test_reference_streams_c2_loop_graphed_deterministic(tmp_path, hip_device, monkeypatch):
    """The same loop with the reference's own streams (rng: python walks, noise: torch) in the
    deterministic mode (DW_DETERMINISTIC=1): the eager run and the run replayed as graphs of 16
    end with bit-identical tables — the float mode's divergence past the first steps above is the
    atomics' order, not the graphs — and leave `random` and torch's generator in the same state."""
    import random
    from tools import train as train_tool
    monkeypatch.setenv('DW_DETERMINISTIC', '1')
    base = ['datamodule.dataset_name=graph_rmat', 'datamodule.additional_parameters.scale=12',
            'datamodule.additional_parameters.n_edges=5429',
            'datamodule.additional_parameters.graph_seed=0',
            'datamodule.additional_parameters.walks_per_node=1',
            'datamodule.additional_parameters.method_params.q=1',
            'datamodule.additional_parameters.rng=python', 'train.noise=torch',
            'model.embedding_size=128', 'train.optimizer.lr=0.01', 'train.max_epochs=2']
    runs = []
    for mode in ('0', '1'):
        monkeypatch.setenv('DW_TRAIN_GRAPH', mode)
        out = str(tmp_path / f'det{mode}')
        random.seed(5)
        torch.manual_seed(0)
        train_tool.main(['--config-name', 'sge_sg_cora', f'path.output_dir={out}',
                         f'output_dir={out}', f'train.experiment=d{mode}'] + base)
        ck = os.path.join(out, 'graph_rmat', f'd{mode}', 'checkpoints', 'last.ckpt')
        runs.append((torch.load(ck, weights_only=True), random.getstate(),
                     torch.get_rng_state()))
    (s0, r0, t0), (s1, r1, t1) = runs
    assert s0['global_step'] == s1['global_step'] == 128
    assert r0 == r1 and torch.equal(t0, t1)
    for k, v in s0['state_dict'].items():
        assert torch.equal(v, s1['state_dict'][k]), k
