"""Analysis of a trained word2vec / graph model (reference: tools/model_analysis.py).

    python tools/model_analysis.py --config-name=w2v_sg_abcde [key=value ...]

Loads ``{output_dir}/{dataset}/{experiment}/checkpoints/{analysis.checkpoint}`` (tools/train.py
output) and, as enabled in the config's ``analysis`` section, writes under
``{output_dir}/{dataset}/{experiment}/analysis/``:
  * closest_pairs.txt — for the ``max_words`` most frequent words (all words when the
    vocabulary is smaller), the ``pairs_per_word`` output-embedding rows closest by cosine
    similarity to the word's input embedding;
  * projected_embeddings.jpg — the input embeddings (t-SNE to 2-D when d > 2, seed 42),
    coloured by label when the dataset has labels;
  * the word-analogy semantics test (Shakespeare-specific, text datasets only) in the log.
Runs on the CPU (no GPU needed to analyse a checkpoint).
"""
import argparse
import logging
import os
import sys
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from shallow_encoders.common.path import CONFIG_PATH  # noqa: E402
from shallow_encoders.config_parser import load_config_dict  # noqa: E402
from shallow_encoders.word2vec.utils.func import pairwise_cosine_similarity  # noqa: E402
from tools import conventions  # noqa: E402
from tools.utils import setup_pipeline  # noqa: E402

logger = logging.getLogger('ModelAnalysis')


def load_tables(checkpoint_path: str):
    """(input, output) embedding tables of a tools/train.py checkpoint (weights-only load)."""
    state = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
    sd = state.get('state_dict', state)
    prefix = '_model.' if '_model._input_embedding.weight' in sd else ''
    return (sd[f'{prefix}_input_embedding.weight'].float(),
            sd[f'{prefix}_output_embedding.weight'].float())


def _sample(dataset, max_words: int) -> List[int]:
    n = len(dataset.vocab)
    if n > max_words:
        return list(dataset.get_n_most_frequent_words(max_words)[1])
    return list(range(n))


def closest_pairs(input_emb: torch.Tensor, output_emb: torch.Tensor, dataset,
                  output_path: Optional[str], max_words: int = 100,
                  pairs_per_word: int = 5) -> Dict[str, List[str]]:
    """{word: its pairs_per_word closest context words} (and closest_pairs.txt)."""
    itos = dataset.vocab.get_itos()
    words = _sample(dataset, max_words)
    sim = pairwise_cosine_similarity(input_emb[words], output_emb)
    top = torch.argsort(sim, dim=1, descending=True)[:, :pairs_per_word]
    result = {itos[w]: [itos[int(j)] for j in top[i]] for i, w in enumerate(words)}
    text = '\n'.join(['Closest pairs in format "{word}:{closest_word_pairs}"'] +
                     [f'{w}: {", ".join(c)}' for w, c in result.items()])
    logger.info(text)
    if output_path:
        path = os.path.join(output_path, 'closest_pairs.txt')
        with open(path, 'w', encoding='utf-8') as f:
            f.write(text)
        logger.info(f'Saved closest pairs analysis result at path "{path}".')
    return result


def visualize_embeddings(input_emb: torch.Tensor, dataset, output_path: str, max_words: int,
                         annotate: bool, skip_unk: bool) -> str:
    """Scatter of the (t-SNE-projected) input embeddings; returns the image path."""
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    emb = input_emb.numpy()
    itos = dataset.vocab.get_itos()
    words = _sample(dataset, max_words)
    if skip_unk:
        words = [w for w in words if w != dataset.vocab['<unk>']]
    pts = emb[words]
    names = [itos[w] for w in words]
    assert pts.shape[1] >= 2, 'Embedding dimension should be 2 or larger.'
    if pts.shape[1] > 2:
        from sklearn.manifold import TSNE
        pts = TSNE(n_components=2, random_state=42,
                   perplexity=min(30.0, max(1.0, len(pts) - 1.0))).fit_transform(pts)
    fig = plt.figure(figsize=(10, 10))
    if dataset.has_labels:
        labels = dataset.labels
        for label in sorted(set(labels.values())):
            ix = [i for i, w in enumerate(names) if labels.get(w) == label]
            plt.scatter(pts[ix, 0], pts[ix, 1], alpha=0.6, label=label)
        plt.legend()
    else:
        plt.scatter(pts[:, 0], pts[:, 1], alpha=0.6)
    if annotate:
        for i, w in enumerate(names):
            plt.annotate(w, (pts[i, 0], pts[i, 1]))
    plt.title('Word Embeddings Visualization')
    plt.xlabel('Dimension 1')
    plt.ylabel('Dimension 2')
    plt.grid(True)
    path = os.path.join(output_path, 'projected_embeddings.jpg')
    fig.savefig(path)
    plt.close(fig)
    logger.info(f'Saved embedding visualization at path "{path}".')
    return path


ANALOGIES = [(['king', 'man', 'woman'], 'queen'), (['queen', 'woman', 'man'], 'king'),
             (['king', 'queen', 'woman'], 'man'), (['queen', 'king', 'man'], 'woman'),
             (['uncle', 'execute', 'kiss'], 'saw')]   # the last one: expected low score


def semantics_test(input_emb: torch.Tensor, output_emb: torch.Tensor, dataset) -> List[float]:
    """vector(a) - vector(b) + vector(c) vs vector(d) (the reference's Shakespeare analogies);
    returns the cosine similarities of the analogies whose words are all in the vocabulary."""
    stoi = dataset.vocab.get_stoi()
    itos = dataset.vocab.get_itos()
    sims = []
    for (a, b, c), d in ANALOGIES:
        if any(w not in stoi for w in (a, b, c, d)):
            logger.warning('Did not find all required words in vocabulary. Skipping....')
            continue
        v = input_emb[stoi[a]] - input_emb[stoi[b]] + input_emb[stoi[c]]
        cos = float(torch.nn.functional.cosine_similarity(v[None], input_emb[stoi[d]][None]))
        sims.append(cos)
        close = torch.argsort(pairwise_cosine_similarity(v[None], output_emb)[0],
                              descending=True)[:5]
        logger.info(f'Similarity between vector("{a}") - vector("{b}") + vector("{c}") and '
                    f'vector("{d}") is {cos:.2f}; closest to it: '
                    f'{", ".join(itos[int(i)] for i in close)}')
    return sims


def parse_args(argv):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument('--config-name', '-cn', default='w2v_sg_abcde')
    ap.add_argument('--config-path', '-cp', default=CONFIG_PATH)
    ap.add_argument('overrides', nargs='*', help='key.sub=value overrides')
    return ap.parse_args(argv)


def main(argv=None) -> Dict[str, object]:
    logging.basicConfig(level=logging.INFO)
    args = parse_args(sys.argv[1:] if argv is None else argv)
    raw = load_config_dict(args.config_name, args.config_path, args.overrides)
    cfg = setup_pipeline(raw, task='analysis')
    dataset = cfg.datamodule.instantiate_dataset()
    out, ds, exp = cfg.path.output_dir, cfg.datamodule.dataset_name, cfg.train.experiment
    w_in, w_out = load_tables(conventions.get_checkpoint_path(out, ds, exp,
                                                              cfg.analysis.checkpoint))
    path = conventions.get_analysis_experiment_path(out, ds, exp)
    Path(path).mkdir(parents=True, exist_ok=True)
    result: Dict[str, object] = {}
    a = cfg.analysis
    if a.closest_pairs.enable:
        result['closest_pairs'] = closest_pairs(w_in, w_out, dataset, path,
                                                a.closest_pairs.max_words,
                                                a.closest_pairs.pairs_per_word)
    if a.visualize_embeddings.enable:
        result['figure'] = visualize_embeddings(w_in, dataset, path,
                                                a.visualize_embeddings.max_words,
                                                a.visualize_embeddings.annotate,
                                                a.visualize_embeddings.skip_unk)
    if a.semantics_test.enable:
        assert not cfg.datamodule.is_graph, 'Semantics test is not supported for graph datasets!'
        result['semantics'] = semantics_test(w_in, w_out, dataset)
    return result


if __name__ == '__main__':
    main()
