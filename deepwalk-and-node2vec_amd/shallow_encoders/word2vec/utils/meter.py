"""Per-epoch metric averaging (reference: word2vec/utils/meter.py:17-83).

Values may stay on the device: the average is computed when the epoch ends, so the training
loop never synchronises per step (the reference moves every loss to the CPU per step).
"""
from collections import defaultdict
from typing import Iterable, Tuple, Union

import torch


class UnknownMetricException(KeyError):
    """No value was pushed for this metric name."""


class MetricMeter:
    """Accumulates metric values and returns their means."""

    def __init__(self):
        self._history = defaultdict(list)

    @property
    def is_empty(self) -> bool:
        return len(self._history) == 0

    def push(self, name: str, value: Union[torch.Tensor, float]) -> None:
        self._history[name].append(value)

    def get(self, name: str) -> Union[torch.Tensor, float]:
        if name not in self._history:
            raise UnknownMetricException(f'Metric name "{name}" not found. '
                                         f'Known metrics: {list(self._history.keys())}.')
        values = self._history[name]
        if values and isinstance(values[0], torch.Tensor):
            return torch.stack([v.reshape(()) for v in values]).mean()
        return sum(values) / len(values)

    def get_all(self, flush: bool = True) -> Iterable[Tuple[str, Union[torch.Tensor, float]]]:
        for name in list(self._history):
            yield name, self.get(name)
        if flush:
            self.flush()

    def flush(self) -> None:
        self._history = defaultdict(list)
