"""Sentence sources of the text datasets (reference: word2vec/dataloader/iterators.py).

Both are re-iterable: ``iter()`` restarts from the first sentence.
"""
from typing import Iterator, List


class InMemoryIterator:
    """Sentences held in a list."""

    def __init__(self, sentences: List[str]):
        self._sentences = list(sentences)

    def __iter__(self) -> Iterator[str]:
        return iter(self._sentences)


class FileIterator:
    """One sentence per line of a UTF-8 text file (opened lazily on each iteration; a missing
    file raises FileNotFoundError when the corpus is first read)."""

    def __init__(self, path: str):
        self._path = path

    def __iter__(self) -> Iterator[str]:
        with open(self._path, 'r', encoding='utf-8') as f:
            yield from f
