"""Corpora -> training batches (reference: word2vec/dataloader/torch_dataset.py:23-322).

``W2VDataset`` is the text corpus: sentences -> tokenize -> vocabulary in
torchtext ``build_vocab_from_iterator`` order -> int64 id tensors per sentence. Lemmatisation
needs nltk's WordNet, which this image lacks: ``lemmatize=True`` raises.

``GraphDataset`` builds the vocabulary straight from the graph — ``<unk>`` = 0, then node
tokens in lexicographic order, the result of the reference's torchtext
``build_vocab_from_iterator`` over one full epoch of walks (torch_dataset.py:91-110; every
node occurs, each counted once). The reference's vocab pass also ADVANCES the global
``random`` stream by one epoch of walks and a reshuffle; ``reference_vocab_pass=True``
reproduces that side effect without generating the walks.

Iteration:
  * ``iter(dataset)`` yields int64 id tensors one walk at a time (the reference's format,
    consumed by ``W2VCollateFunctional`` in a torch ``DataLoader``);
  * ``walk_batches(batch_size)`` yields device int32 [n, L] walk batches straight from the
    gfx950 walker — the hot path (no strings, no host windows).
"""
import logging
import re
from collections import Counter
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import IterableDataset

from shallow_encoders.graph.datasets import RandomWalkDataset
from shallow_encoders.graph.rng import skip_uniforms
from shallow_encoders.word2vec.dataloader import w2v_datasets  # noqa: F401 (registers corpora)
from shallow_encoders.word2vec.dataloader.registry import DATASET_REGISTRY

logger = logging.getLogger('W2VDataset')

_TOKEN_RE = re.compile(r"[A-Za-z]+[\w^']*|[\w^']*[A-Za-z]+[\w^']*|<unk>")


def tokenize(text: str) -> List[str]:
    """Lower-case, keep word-like tokens and ``<unk>`` (torch_dataset.py:23-39)."""
    return _TOKEN_RE.findall(text.lower())


class Vocab:
    """The slice of torchtext's Vocab API the reference uses (default index = ``<unk>``)."""

    def __init__(self, itos: List[str]):
        self._itos = list(itos)
        self._stoi = {t: i for i, t in enumerate(self._itos)}
        self._default = self._stoi.get('<unk>', 0)

    def __len__(self) -> int:
        return len(self._itos)

    def __contains__(self, token: str) -> bool:
        return token in self._stoi

    def __getitem__(self, token: str) -> int:
        return self._stoi.get(token, self._default)

    def __call__(self, tokens: List[str]) -> List[int]:
        return [self[t] for t in tokens]

    def lookup_token(self, index: int) -> str:
        return self._itos[index]

    def lookup_tokens(self, indices: List[int]) -> List[str]:
        return [self._itos[i] for i in indices]

    def get_itos(self) -> List[str]:
        return list(self._itos)

    def get_stoi(self) -> Dict[str, int]:
        return dict(self._stoi)

    def set_default_index(self, index: int) -> None:
        self._default = index


def build_vocab(token_lists: Iterable[List[str]], specials: List[str], min_freq: int) -> Vocab:
    """torchtext 0.15 ``build_vocab_from_iterator`` order (pinned version of the reference's
    requirements; torchtext itself is absent here): specials first, then the other tokens with
    frequency >= min_freq by descending frequency, ties alphabetical."""
    counter: Counter = Counter()
    for tokens in token_lists:
        counter.update(tokens)
    for sp in specials:
        counter.pop(sp, None)
    ordered = sorted(counter.items(), key=lambda kv: (-kv[1], kv[0]))
    return Vocab(list(specials) + [t for t, f in ordered if f >= min_freq])


class W2VDataset(IterableDataset):
    """Text word2vec corpus (torch_dataset.py:61-213): iterates sentences as int64 id tensors.

    Sentences shorter than 2R+1 tokens are dropped (not counted for the vocabulary filter
    either way: the vocabulary pass reads every sentence, the iteration skips short ones).
    """

    def __init__(self, dataset_name: str, context_radius: int = 5, min_word_frequency: int = 20,
                 lemmatize: bool = False, sort_by_frequency: bool = True,
                 additional_parameters: Optional[dict] = None):
        assert dataset_name in DATASET_REGISTRY, \
            f'Dataset "{dataset_name}" is not supported. Supported: {list(DATASET_REGISTRY.keys())}'
        if lemmatize:
            raise NotImplementedError('lemmatize=True needs nltk WordNet (not in this image)')
        self._context_radius = context_radius
        self._dataset = DATASET_REGISTRY[dataset_name](**(additional_parameters or {}))
        token_lists = list(self.get_iterator(apply_filter=False))
        if sort_by_frequency:
            vocab_source = token_lists
        else:  # every token counted once: alphabetical order after the specials
            vocab_source = [[t] for t in {t for tokens in token_lists for t in tokens}]
        self._vocab = build_vocab(vocab_source, ['<unk>'], min_word_frequency)
        logger.info(f'Vocabulary size: {len(self._vocab)}')
        freq: Counter = Counter()
        for tokens in token_lists:
            freq.update(t for t in tokens if t in self._vocab)
        self._word_frequency = dict(freq)

    def sentence_pipeline(self, sentence: str, apply_filter: bool = True) -> Optional[List[str]]:
        tokens = tokenize(sentence)
        if apply_filter and len(tokens) < 2 * self._context_radius + 1:
            return None
        return tokens

    def get_iterator(self, apply_filter: bool = True) -> Iterator[List[str]]:
        for sentence in self._dataset:
            tokens = self.sentence_pipeline(sentence, apply_filter=apply_filter)
            if tokens is not None:
                yield tokens

    def get_n_most_frequent_words(self, n: int) -> Tuple[List[str], List[int]]:
        """The n most frequent vocabulary words (ties in first-occurrence order) and their ids."""
        words = [w for w, _ in sorted(self._word_frequency.items(), key=lambda x: x[1],
                                      reverse=True)[:n]]
        return words, [self._vocab[w] for w in words]

    @property
    def vocab(self) -> Vocab:
        return self._vocab

    @property
    def context_radius(self) -> int:
        return self._context_radius

    @property
    def has_labels(self) -> bool:
        return False

    @property
    def labels(self) -> Dict[str, str]:
        raise NotImplementedError('This function is not implemented!')

    @property
    def has_features(self) -> bool:
        return False

    def __iter__(self) -> Iterator[torch.Tensor]:
        for tokens in self.get_iterator():
            yield torch.tensor(self._vocab(tokens), dtype=torch.long)


class GraphDataset(IterableDataset):
    """Graph random-walk corpus (torch_dataset.py:216-273)."""

    def __init__(self, dataset_name: str, context_radius: int = 5,
                 additional_parameters: Optional[dict] = None,
                 reference_vocab_pass: bool = False):
        assert dataset_name in DATASET_REGISTRY, \
            f'Dataset "{dataset_name}" is not supported. Supported: {list(DATASET_REGISTRY.keys())}'
        additional_parameters = {} if additional_parameters is None else dict(additional_parameters)
        self._context_radius = context_radius
        self._dataset = DATASET_REGISTRY[dataset_name](**additional_parameters)
        assert isinstance(self._dataset, RandomWalkDataset), \
            f'Expected RandomWalkDataset dataset but got {type(self._dataset)}!'
        csr = self._dataset.csr
        self._vocab = Vocab(csr.itos)
        logger.info(f'Vocabulary size: {len(self._vocab)}')
        if reference_vocab_pass:
            # the reference generates one epoch of walks (one double per step) to build the
            # vocabulary, then reshuffles the start nodes at StopIteration
            steps = len(self._dataset) * max(self._dataset.walk_length - 1, 0)
            skip_uniforms(steps)
            self._dataset._reshuffle()  # noqa: SLF001
        self._word_frequency = None
        self._pipeline_state = None

    # ---- reference surface -----------------------------------------------------------------
    @property
    def vocab(self) -> Vocab:
        return self._vocab

    @property
    def context_radius(self) -> int:
        return self._context_radius

    @property
    def dataset(self) -> RandomWalkDataset:
        return self._dataset

    @property
    def has_labels(self) -> bool:
        return self._dataset.has_labels

    @property
    def labels(self) -> Dict[str, str]:
        return self._dataset.labels

    @property
    def has_features(self) -> bool:
        return self._dataset.has_features

    @property
    def features(self) -> Dict[str, np.ndarray]:
        return self._dataset.features

    @property
    def graph(self):
        return self._dataset.graph

    def get_n_most_frequent_words(self, n: int) -> Tuple[List[str], List[int]]:
        """The n most frequent nodes. The reference counts node visits over its random vocabulary
        epoch of walks (torch_dataset.py:113-119); a walk visits a node about in proportion to its
        degree, so the deterministic order here is descending degree (ties by id)."""
        deg = np.diff(self._dataset.csr.row_ptr)
        deg[0] = -1                                    # never <unk>
        ids = np.lexsort((np.arange(len(deg)), -deg))[:min(n, len(deg) - 1)]
        return [self._vocab.lookup_token(int(i)) for i in ids], [int(i) for i in ids]

    def sentence_pipeline(self, sentence: str, apply_filter: bool = True) -> Optional[List[str]]:
        tokens = tokenize(sentence)
        if apply_filter and len(tokens) < 2 * self._context_radius + 1:
            return None
        return tokens

    def __iter__(self) -> 'GraphDataset':
        self._pipeline_state = iter(self._dataset)
        return self

    def __next__(self) -> torch.Tensor:
        while True:
            tokens = self.sentence_pipeline(next(self._pipeline_state))
            if tokens is not None:
                return torch.tensor(self._vocab(tokens), dtype=torch.long)

    # ---- device batches (hot path) -----------------------------------------------------------
    def walk_batches(self, batch_size: int, check: bool = False) -> Iterator[torch.Tensor]:
        """One epoch of device walk batches int32 [<=batch_size, L] (reshuffles at the end)."""
        if self._dataset.walk_length < 2 * self._context_radius + 1:
            # every walk would be filtered out by sentence_pipeline (torch_dataset.py:154)
            while self._dataset.next_walk_batch(batch_size, check=check) is not None:
                pass
            return
        while True:
            b = self._dataset.next_walk_batch(batch_size, check=check)
            if b is None:
                return
            yield b


class W2VCollateFunctional:
    """Batch collation for 'sg' / 'cbow' (torch_dataset.py:276-322), vectorised with unfold.

    For each text (clipped to max_length) and centre i in [R, len-R):
      sg:   inputs = text[i:i+1], targets = text[i-R:i] | text[i+1:i+1+R]
      cbow: the two swapped. Output rows follow text order, then centre order.
    """

    def __init__(self, mode: str, context_radius: int, max_length: int):
        assert mode.lower() in ['sg', 'cbow'], 'Invalid collate mode! Choose "sg" or "cbow"!'
        self._mode = mode.lower()
        self._context_radius = context_radius
        self._min_text_length = 2 * context_radius + 1
        self._max_length = max_length

    def __call__(self, batch_text: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        R = self._context_radius
        centres, contexts = [], []
        for text in batch_text:
            text = text[:self._max_length]
            text_length = text.shape[0]
            assert text_length >= self._min_text_length, \
                f'Text is too short! [{text_length=}] < [{self._min_text_length=}]'
            win = text.unfold(0, 2 * R + 1, 1)                  # (len-2R, 2R+1)
            centres.append(win[:, R:R + 1])
            contexts.append(torch.cat([win[:, :R], win[:, R + 1:]], dim=1))
        c = torch.cat(centres, dim=0)
        ctx = torch.cat(contexts, dim=0)
        if self._mode == 'sg':
            return c, ctx
        return ctx, c
