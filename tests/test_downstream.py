"""Downstream quality harness: split algorithms and edge operators against
fixtures recorded from the reference (tests/golden/make_golden.py downstream), and the node /
edge classification tasks of tools/graph_model_downstream_classification.py on synthetic
embeddings (CPU; the trained-embedding run is in test_gpu_trainer.py)."""
import os
import random

import networkx as nx
import numpy as np
import pytest

from conftest import golden

SPLIT_CASES = [  # must match tests/golden/make_golden.py
    ('TrainTestRatioSplit', {'train_ratio': 0.5}),
    ('TrainTestRatioSplit', {'train_ratio': 0.7, 'stratify': True}),
    ('TrainTestRatioSplit', {'train_ratio': 0.5, 'test_all': True}),
    ('TrainValTestRatioSplit', {'train_ratio': 0.6, 'val_ratio': 0.8}),
    ('TrainValTestRatioSplit', {'train_ratio': 0.5, 'val_ratio': 0.7, 'stratify': True}),
    ('TrainValTestStratifiedNSamplesSplit', {'train_samples': 3, 'val_samples': 2,
                                             'test_samples': 4}),
    ('TrainValTestStratifiedNSamplesSplit', {'train_samples': 3, 'val_samples': 2}),
]


@pytest.mark.parametrize('case', range(len(SPLIT_CASES)))
def test_split_algorithms_match_reference(case):
    import shallow_encoders.split as split
    f = golden('downstream_split_ops.npz')
    cls, kw = SPLIT_CASES[case]
    for seed in (0, 7, 42):
        algo = getattr(split, cls)(**kw)
        algo.random_state = seed
        out = algo(f['X'], f['y'])
        keys = sorted(k[len(f'split{case}_seed{seed}_'):] for k in f.files
                      if k.startswith(f'split{case}_seed{seed}_'))
        assert sorted(out) == keys
        for k in keys:
            np.testing.assert_array_equal(out[k], f[f'split{case}_seed{seed}_{k}'])


def test_stratified_n_samples_rejects_small_classes():
    from shallow_encoders.split import TrainValTestStratifiedNSamplesSplit
    X, y = np.zeros((6, 2)), np.asarray([0, 0, 0, 1, 1, 1], dtype=np.float32)
    with pytest.raises(AssertionError):
        TrainValTestStratifiedNSamplesSplit(2, 2)(X, y)


def test_edge_operators_match_reference():
    from shallow_encoders.graph import edge_operators as ops
    f = golden('downstream_split_ops.npz')
    for name in ('average', 'hadamard', 'weighted_l1', 'weighted_l2'):
        op = ops.edge_operator_factory(name.upper())
        np.testing.assert_allclose(op(f['op_lhs'], f['op_rhs']), f[f'op_{name}'], rtol=0,
                                   atol=1e-15)
        emb = np.concatenate([f['op_lhs'], f['op_rhs']])
        pairs = np.stack([np.arange(6), np.arange(6) + 6], axis=1)
        np.testing.assert_allclose(ops.edge_embeddings(emb, pairs, op), f[f'op_{name}'],
                                   atol=1e-15)
    with pytest.raises(AssertionError):
        ops.edge_operator_factory('cosine')


def test_default_split_algorithm_is_usable():
    from shallow_encoders.config_parser.core import GraphDownstreamNodeClassificationConfig
    from shallow_encoders.split import TrainTestRatioSplit
    algo = GraphDownstreamNodeClassificationConfig().instantiate_split_algorithm()
    assert isinstance(algo, TrainTestRatioSplit) and algo.random_state == 42
    out = algo(np.zeros((10, 2)), np.arange(10, dtype=np.float32))
    assert len(out['X_train']) == 5


def test_node_classification_on_separable_embeddings():
    from shallow_encoders.split import TrainTestRatioSplit
    from tools.graph_model_downstream_classification import node_classification
    g = nx.karate_club_graph()
    itos = ['<unk>'] + sorted(f'n{i:02d}' for i in range(34))
    labels = {f'n{i:02d}': g.nodes[i]['club'] for i in range(34)}
    rng = np.random.default_rng(0)
    centre = {'Mr. Hi': np.array([2.0, 0.0]), 'Officer': np.array([-2.0, 0.0])}
    emb = np.zeros((35, 2))
    for i, v in enumerate(itos[1:], start=1):
        emb[i] = centre[labels[v]] + 0.3 * rng.normal(size=2)
    mean, best = node_classification(emb, itos, labels, TrainTestRatioSplit(0.5, test_all=True),
                                     n_experiments=5)
    assert mean == 1.0 and best == 1.0


def test_edge_classification_and_negative_sampler():
    from tools.graph_model_downstream_classification import (edge_classification,
                                                             sample_negative_edges)
    g = nx.relabel_nodes(nx.karate_club_graph(), {i: f'n{i:02d}' for i in range(34)})
    nodes = list(g.nodes)
    nbrs = {u: set(g.neighbors(u)) for u in nodes}
    neg = sample_negative_edges(nodes, nbrs, 500, random.Random(1))
    assert len(neg) == 500 and all(v not in nbrs[u] for u, v in neg)
    stoi = {v: i + 1 for i, v in enumerate(sorted(nodes))}
    emb = np.random.default_rng(2).normal(size=(35, 8))
    mean, best = edge_classification(emb, g, stoi, 0.5, 5, 'hadamard')
    assert 0.0 <= mean <= best <= 1.0


def test_text_corpus_vocab_and_ids_like_reference_run_test():
    """The reference's only test-like code, torch_dataset.py:323-336 run_test():
    W2VDataset('test', min_word_frequency=2, context_radius=1). Expected values follow
    torchtext 0.15's build_vocab_from_iterator rule (specials first, then by descending
    frequency, ties alphabetical; torchtext itself is not importable here, so the rule — not
    its code — pins this) and the collate length filter (2R + 1 = 3 tokens)."""
    from shallow_encoders.word2vec.dataloader.torch_dataset import W2VDataset
    ds = W2VDataset(dataset_name='test', min_word_frequency=2, context_radius=1)
    assert ds.vocab.get_itos() == ['<unk>', 'a', 'b', 'hello', 'here', 'test', 'there', 'world']
    assert [t.tolist() for t in ds] == [[1, 1, 0, 2, 2], [3, 7, 3, 7], [5, 4, 5, 6, 4, 6]]
    assert ds.get_n_most_frequent_words(2) == (['a', 'b'], [1, 2])


def test_model_analysis_tool(tmp_path):
    """tools/model_analysis.py on a checkpoint: closest pairs (cosine of input rows vs output
    rows), the projected-embedding figure (t-SNE when d > 2) and the graph dataset's
    most-frequent order (by degree)."""
    import torch
    from shallow_encoders.config_parser import load_config
    from tools import conventions
    from tools import model_analysis
    out = str(tmp_path / 'runs')
    cfg = load_config('sge_sg_karate_club', overrides=[f'path.output_dir={out}'])
    ds = cfg.datamodule.instantiate_dataset()
    V = len(ds.vocab)
    rng = np.random.default_rng(0)
    w_in, w_out = rng.normal(size=(V, 4)).astype(np.float32), rng.normal(size=(V, 4))
    w_out = w_out.astype(np.float32)
    w_out[5] = w_in[3] * 2.0                     # word 3's closest context word is 5
    ck = conventions.get_checkpoint_path(out, cfg.datamodule.dataset_name, cfg.train.experiment,
                                         'last.ckpt')
    os.makedirs(os.path.dirname(ck))
    torch.save({'state_dict': {'_model._input_embedding.weight': torch.from_numpy(w_in),
                               '_model._output_embedding.weight': torch.from_numpy(w_out)}}, ck)
    res = model_analysis.main(['--config-name', 'sge_sg_karate_club', f'path.output_dir={out}',
                               f'output_dir={out}'])
    itos = ds.vocab.get_itos()
    assert res['closest_pairs'][itos[3]][0] == itos[5]
    assert os.path.exists(res['figure'])
    words, ids = ds.get_n_most_frequent_words(3)
    deg = np.diff(ds.dataset.csr.row_ptr)
    assert list(ids) == sorted(range(1, V), key=lambda i: (-deg[i], i))[:3]
    assert words == [itos[i] for i in ids]
