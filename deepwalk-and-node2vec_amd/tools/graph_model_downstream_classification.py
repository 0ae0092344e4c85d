"""Downstream quality of trained graph embeddings (reference:
tools/graph_model_downstream_classification.py; README.md:225-248, 276-281, 320-325).

    python tools/graph_model_downstream_classification.py --config-name=sge_sg_karate_club

Loads ``{output_dir}/{dataset}/{experiment}/checkpoints/{analysis.checkpoint}`` (written by
tools/train.py) and runs the two tasks of the reference:
  * node classification: logistic regression on the input embeddings (``<unk>`` row skipped,
    node features appended when the dataset has them); the configured split algorithm is
    re-seeded with the experiment index; mean and best accuracy over ``n_experiments``;
  * edge classification (link prediction): edge embedding = operator(n1, n2); per
    experiment the edges are shuffled, the first round(train_ratio * E) are the positive
    training edges, as many negative (non-adjacent) pairs are sampled for training and the rest
    for evaluation; the classifier is evaluated on ALL edges plus both negative sets
    (transductive, as the reference does).
Negative pairs follow the reference's law: a uniform node, then a uniform node among its
non-neighbours (itself included). sklearn's LogisticRegression with the config's
``classifier_params``. The model only needs the checkpoint: no GPU is used here.
"""
import argparse
import logging
import os
import random
import sys
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from shallow_encoders.common.path import CONFIG_PATH  # noqa: E402
from shallow_encoders.config_parser import load_config_dict  # noqa: E402
from shallow_encoders.graph import edge_operators  # noqa: E402
from tools import conventions  # noqa: E402
from tools.utils import setup_pipeline  # noqa: E402

logger = logging.getLogger('DownstreamTask-Classification')


def labels_to_integers(labels: List[str]) -> List[int]:
    """Unique string labels -> 0..C-1 (sorted order, so runs are reproducible)."""
    index = {label: i for i, label in enumerate(sorted(set(labels)))}
    return [index[label] for label in labels]


def fit_and_score(X_train, y_train, X, y, classifier_params: Optional[dict] = None):
    """LogisticRegression fitted on (X_train, y_train); accuracy on (X, y)."""
    from sklearn.linear_model import LogisticRegression
    clf = LogisticRegression(**(classifier_params or {}))
    clf.fit(X_train, y_train)
    return clf, float(np.mean(clf.predict(X) == y))


def node_classification(embeddings: np.ndarray, itos: List[str], labels: Dict[str, str],
                        split_algorithm, n_experiments: int,
                        features: Optional[Dict[str, np.ndarray]] = None,
                        classifier_params: Optional[dict] = None,
                        plot_path: Optional[str] = None) -> Tuple[float, float]:
    """Mean and best accuracy over ``n_experiments`` (rows of ``embeddings`` follow ``itos``,
    row 0 = ``<unk>`` is skipped)."""
    vertices = itos[1:]
    X = np.asarray(embeddings, dtype=np.float64)[1:]
    if features is not None:
        X = np.concatenate([X, np.stack([features[v] for v in vertices])], axis=1)
    y = np.asarray(labels_to_integers([labels[v] for v in vertices]), dtype=np.float32)
    logger.info(f'Dataset info: X.shape={X.shape}, y.shape={y.shape}.')
    total, best, best_clf = 0.0, None, None
    for i in range(n_experiments):
        split_algorithm.random_state = i
        sp = split_algorithm(X, y)
        clf, acc = fit_and_score(sp['X_train'], sp['y_train'], sp['X_test'], sp['y_test'],
                                 classifier_params)
        total += acc
        if best is None or acc >= best:
            best, best_clf = acc, clf
    assert best is not None, 'No experiments performed!'
    mean = total / n_experiments
    logger.info(f'Node classification accuracy: {100 * mean:.2f}% (averaged over '
                f'{n_experiments} experiments); best {100 * best:.2f}%.')
    if plot_path is not None:
        plot_node_classification(X, y, best_clf, best, plot_path)
    return mean, best


def plot_node_classification(X, y, clf, accuracy, path) -> None:
    """Scatter of 2-D embeddings per class with the classifier's decision lines."""
    if X.shape[1] != 2:
        logger.info('Embeddings are not 2-D: skipping the decision-boundary figure.')
        return
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(10, 10))
    for c in np.unique(y):
        pts = X[y == c]
        plt.scatter(pts[:, 0], pts[:, 1], label=f'class {int(c)}')
    xs = np.linspace(X[:, 0].min() - 1, X[:, 0].max() + 1, 100)
    for i in range(clf.coef_.shape[0]):
        t1, t2 = clf.coef_[i]
        plt.plot(xs, (-clf.intercept_[i] - t1 * xs) / t2, color='red',
                 label=f'Decision Boundary {i:03d}')
    plt.title(f'Classification on embeddings - Accuracy {100 * accuracy:.2f}')
    plt.xlabel('Dimension 1')
    plt.ylabel('Dimension 2')
    plt.legend()
    fig.savefig(path)
    plt.close(fig)
    logger.info(f'Saved figure at path "{path}".')


def sample_negative_edges(nodes: List[str], neighbors: Dict[str, set], n: int,
                          rng: random.Random) -> List[Tuple[str, str]]:
    """``n`` pairs (u, v): u uniform over nodes, v uniform over the nodes not adjacent to u
    (u itself allowed) — drawn by rejection, the same law as the reference's set difference."""
    out = []
    node_set_size = len(nodes)
    while len(out) < n:
        u = rng.choice(nodes)
        if len(neighbors[u]) >= node_set_size:
            continue
        while True:
            v = rng.choice(nodes)
            if v not in neighbors[u]:
                break
        out.append((u, v))
    return out


def edge_classification(embeddings: np.ndarray, graph, stoi: Dict[str, int], train_ratio: float,
                        n_experiments: int, operator_name: str,
                        classifier_params: Optional[dict] = None,
                        seed: int = 0) -> Tuple[float, float]:
    """Mean and best link-prediction accuracy over ``n_experiments``."""
    op = edge_operators.edge_operator_factory(operator_name)
    emb = np.asarray(embeddings, dtype=np.float64)
    edges = list(graph.edges)
    nodes = list(graph.nodes)
    neighbors = {u: set(graph.neighbors(u)) for u in nodes}
    n_edges = len(edges)
    rng = random.Random(seed)

    def ids(pairs):
        return np.asarray([(stoi[a], stoi[b]) for a, b in pairs], dtype=np.int64).reshape(-1, 2)

    total, best = 0.0, None
    for _ in range(n_experiments):
        n_train = round(train_ratio * n_edges)
        n_val = n_edges - n_train
        rng.shuffle(edges)
        neg_train = sample_negative_edges(nodes, neighbors, n_train, rng)
        neg_val = sample_negative_edges(nodes, neighbors, n_val, rng)
        X_train = edge_operators.edge_embeddings(emb, ids(edges[:n_train] + neg_train), op)
        y_train = np.asarray([1] * n_train + [0] * n_train, dtype=np.float32)
        X = edge_operators.edge_embeddings(emb, ids(edges + neg_train + neg_val), op)
        y = np.asarray([1] * n_edges + [0] * (n_train + n_val), dtype=np.float32)
        _, acc = fit_and_score(X_train, y_train, X, y, classifier_params)
        total += acc
        best = acc if best is None else max(best, acc)
    assert best is not None, 'No experiments performed!'
    mean = total / n_experiments
    logger.info(f'Edge classification accuracy: {100 * mean:.2f}% (averaged over '
                f'{n_experiments} experiments); best {100 * best:.2f}%.')
    return mean, best


def load_input_embeddings(cfg, dataset, checkpoint_path: str) -> np.ndarray:
    """Input-embedding table of a tools/train.py checkpoint (weights-only load)."""
    import torch
    state = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
    sd = state.get('state_dict', state)
    key = '_model._input_embedding.weight'
    if key not in sd:
        key = '_input_embedding.weight'
    w = sd[key].numpy()
    assert w.shape[0] == len(dataset.vocab), \
        f'checkpoint has {w.shape[0]} rows, the dataset vocabulary {len(dataset.vocab)}'
    return w


def parse_args(argv):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument('--config-name', '-cn', default='sge_sg_graph_triplets')
    ap.add_argument('--config-path', '-cp', default=CONFIG_PATH)
    ap.add_argument('overrides', nargs='*', help='key.sub=value overrides')
    return ap.parse_args(argv)


def main(argv=None) -> Dict[str, float]:
    logging.basicConfig(level=logging.INFO)
    args = parse_args(sys.argv[1:] if argv is None else argv)
    raw = load_config_dict(args.config_name, args.config_path, args.overrides)
    cfg = setup_pipeline(raw, task='downstream-classification')
    assert cfg.datamodule.is_graph, 'This script supports only graph datasets!'
    dataset = cfg.datamodule.instantiate_dataset()
    out, ds, exp = cfg.path.output_dir, cfg.datamodule.dataset_name, cfg.train.experiment
    ckpt = conventions.get_checkpoint_path(out, ds, exp, cfg.analysis.checkpoint)
    emb = load_input_embeddings(cfg, dataset, ckpt)
    analysis_dir = conventions.get_analysis_experiment_path(out, ds, exp)
    Path(analysis_dir).mkdir(parents=True, exist_ok=True)
    result: Dict[str, float] = {}
    nc = cfg.downstream.node_classification
    if nc.enable:
        plot = os.path.join(analysis_dir, 'downstream-node-classification.jpg') \
            if nc.visualize else None
        result['node_accuracy'], result['node_best'] = node_classification(
            emb, dataset.vocab.get_itos(), dataset.labels, nc.instantiate_split_algorithm(),
            nc.n_experiments, features=dataset.features if dataset.has_features else None,
            classifier_params=nc.classifier_params, plot_path=plot)
    ec = cfg.downstream.edge_classification
    if ec.enable:
        result['edge_accuracy'], result['edge_best'] = edge_classification(
            emb, dataset.graph, dataset.vocab.get_stoi(), ec.train_ratio, ec.n_experiments,
            ec.operator_name, classifier_params=ec.classifier_params)
    print(' '.join(f'{k}={100 * v:.2f}%' for k, v in result.items()), flush=True)
    return result


if __name__ == '__main__':
    main()
