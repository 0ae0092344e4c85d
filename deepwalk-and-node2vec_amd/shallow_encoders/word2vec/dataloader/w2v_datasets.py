"""Text corpora for word2vec (reference: word2vec/dataloader/w2v_datasets.py).

Registered under the reference's names: ``test`` and ``abcde`` (in memory), ``wiki-text-2`` /
``wiki-text-103`` ({assets}/wikitext-*/wiki.train.tokens, one sentence per line) and
``shakespeare`` ({assets}/Shakespeare_data.csv, column PlayerLine). The file-backed corpora are
not shipped (no network here): constructing a W2VDataset over them raises FileNotFoundError.
"""
import os

from shallow_encoders.common.path import ASSETS_PATH
from shallow_encoders.word2vec.dataloader.iterators import FileIterator, InMemoryIterator
from shallow_encoders.word2vec.dataloader.registry import register_dataset


@register_dataset('test')
class TestDataset(InMemoryIterator):
    """Tiny corpus for dataloader tests."""

    def __init__(self):
        super().__init__(['a, a, c, b, b', 'hello world! hello world!',
                          'test here, test there, here there', '.'])


@register_dataset('abcde')
class ABCDEDataset(InMemoryIterator):
    """Toy corpus: `a` co-occurs with `b`, `c` with `d`, `e` only with itself."""

    def __init__(self):
        super().__init__([
            'a b a b a b a b a b', 'a b a b a b', 'b a b a', 'a b a b a b a b',
            'c d c d c d c d', 'd c d c d c', 'c d c d c d',
            'e e e e e e e e', 'e e e',
        ])


class WikiTextDataset(FileIterator):
    """{assets}/{name}/wiki.{split}.tokens."""

    def __init__(self, dataset_name: str, split: str = 'train', assets_path: str = ASSETS_PATH):
        super().__init__(os.path.join(assets_path, dataset_name, f'wiki.{split}.tokens'))


@register_dataset('wiki-text-2')
class WikiText2Dataset(WikiTextDataset):
    def __init__(self, assets_path: str = ASSETS_PATH):
        super().__init__('wikitext-2', 'train', assets_path)


@register_dataset('wiki-text-103')
class WikiText103Dataset(WikiTextDataset):
    def __init__(self, assets_path: str = ASSETS_PATH):
        super().__init__('wikitext-103', 'train', assets_path)


@register_dataset('shakespeare')
class ShakespeareDataset(InMemoryIterator):
    """Player lines of {assets}/Shakespeare_data.csv."""

    def __init__(self, assets_path: str = ASSETS_PATH):
        import pandas as pd
        path = os.path.join(assets_path, 'Shakespeare_data.csv')
        if not os.path.exists(path):
            raise FileNotFoundError(f'Shakespeare corpus not found at "{path}"')
        super().__init__(pd.read_csv(path)['PlayerLine'].astype(str).tolist())
