"""Dataset plugin registry (reference: word2vec/dataloader/registry.py:6-26).

``@register_dataset(name)`` adds a class to ``DATASET_REGISTRY``; datasets are constructed with
``**datamodule.additional_parameters`` (torch_dataset.py:89).
"""
from typing import Callable, Type

DATASET_REGISTRY = {}


def register_dataset(name: str) -> Callable[[Type], Type]:
    """Class decorator registering a dataset under ``name`` (names are unique)."""
    assert name not in DATASET_REGISTRY, f'Already registered "{name}"!'

    def decorator(cls: Type) -> Type:
        DATASET_REGISTRY[name] = cls
        return cls

    return decorator
