"""Split algorithms of the downstream tasks (reference: shallow_encoders/split/core.py).

Same constructor arguments, seeds and outputs as the reference so a config's split reproduces
the same partitions:
  * TrainTestRatioSplit       sklearn ``train_test_split`` with test_size = 1 - train_ratio
                              (optionally stratified; ``test_all`` evaluates on everything);
  * TrainValTestRatioSplit    two chained ``train_test_split`` calls, the second with
                              test_size = (1 - val_ratio) / (1 - train_ratio);
  * TrainValTestStratifiedNSamplesSplit
                              per class (``np.unique`` order): the numpy global generator is
                              seeded with ``random_state`` and the class's indices shuffled in
                              place, then the first train / val / test samples are taken.
All of them return dicts of copies keyed X_train / y_train / [X_val / y_val /] X_test / y_test.
"""
from abc import ABC, abstractmethod
from typing import Dict, List, Optional

import numpy as np
from sklearn.model_selection import train_test_split

DEFAULT_RANDOM_STATE = 42


class SplitAlgorithm(ABC):
    """Callable split: ``algo(X, y) -> dict``; ``random_state`` is settable per experiment."""

    def __init__(self, random_state: Optional[int] = None):
        self._random_state = DEFAULT_RANDOM_STATE if random_state is None else random_state

    @property
    def random_state(self) -> int:
        return self._random_state

    @random_state.setter
    def random_state(self, random_state: int) -> None:
        self._random_state = random_state

    @abstractmethod
    def split(self, X: np.ndarray, y: np.ndarray) -> Dict[str, np.ndarray]:
        """Partition (X, y)."""

    def __call__(self, X: np.ndarray, y: np.ndarray) -> Dict[str, np.ndarray]:
        return self.split(X, y)


def _copies(**parts: np.ndarray) -> Dict[str, np.ndarray]:
    return {k: v.copy() for k, v in parts.items()}


class TrainTestRatioSplit(SplitAlgorithm):
    """Train / test by ratio; ``stratify`` keeps class proportions; ``test_all`` returns the whole
    data as the test split (transductive evaluation, as the graph configs use)."""

    def __init__(self, train_ratio: float, stratify: bool = False, test_all: bool = False,
                 random_state: Optional[int] = None):
        super().__init__(random_state=random_state)
        self._train_ratio = train_ratio
        self._stratify = stratify
        self._test_all = test_all

    def split(self, X: np.ndarray, y: np.ndarray) -> Dict[str, np.ndarray]:
        X_tr, X_te, y_tr, y_te = train_test_split(
            X, y, test_size=1 - self._train_ratio, stratify=y if self._stratify else None,
            random_state=self._random_state)
        if self._test_all:
            X_te, y_te = X, y
        return _copies(X_train=X_tr, y_train=y_tr, X_test=X_te, y_test=y_te)


class TrainValTestRatioSplit(SplitAlgorithm):
    """Train / (val + test) by ``train_ratio``, then val / test with the reference's second
    test fraction (1 - val_ratio) / (1 - train_ratio)."""

    def __init__(self, train_ratio: float, val_ratio: float, stratify: bool = False,
                 random_state: Optional[int] = None):
        super().__init__(random_state=random_state)
        self._train_ratio = train_ratio
        self._val_ratio = val_ratio
        self._stratify = stratify

    def split(self, X: np.ndarray, y: np.ndarray) -> Dict[str, np.ndarray]:
        X_tr, X_rest, y_tr, y_rest = train_test_split(
            X, y, test_size=1 - self._train_ratio, stratify=y if self._stratify else None,
            random_state=self._random_state)
        X_va, X_te, y_va, y_te = train_test_split(
            X_rest, y_rest, test_size=(1 - self._val_ratio) / (1 - self._train_ratio),
            stratify=y_rest if self._stratify else None, random_state=self._random_state)
        return _copies(X_train=X_tr, y_train=y_tr, X_val=X_va, y_val=y_va, X_test=X_te,
                       y_test=y_te)


class TrainValTestStratifiedNSamplesSplit(SplitAlgorithm):
    """A fixed number of samples per class for train and val (and optionally test; otherwise
    the rest of the class). Raises AssertionError when a class is too small."""

    def __init__(self, train_samples: int, val_samples: int, test_samples: Optional[int] = None,
                 random_state: Optional[int] = None):
        super().__init__(random_state=random_state)
        self._n_train = train_samples
        self._n_val = val_samples
        self._n_test = test_samples

    def split(self, X: np.ndarray, y: np.ndarray) -> Dict[str, np.ndarray]:
        np.random.seed(self._random_state)
        classes = np.unique(y)
        parts: Dict[str, List[int]] = {'train': [], 'val': [], 'test': []}
        a, b = self._n_train, self._n_train + self._n_val
        for label in classes:
            idx = np.where(y == label)[0]
            np.random.shuffle(idx)
            parts['train'].extend(idx[:a])
            parts['val'].extend(idx[a:b])
            parts['test'].extend(idx[b:] if self._n_test is None else idx[b:b + self._n_test])
        k = classes.shape[0]
        expect = {'train': k * self._n_train, 'val': k * self._n_val}
        if self._n_test is not None:
            expect['test'] = k * self._n_test
        for name, n in expect.items():
            assert len(parts[name]) == n, f'{len(parts[name])} != {n}'
        out = {}
        for name in ('train', 'val', 'test'):
            ix = np.asarray(parts[name], dtype=np.int64)
            out[f'X_{name}'], out[f'y_{name}'] = X[ix], y[ix]
        return _copies(**out)
