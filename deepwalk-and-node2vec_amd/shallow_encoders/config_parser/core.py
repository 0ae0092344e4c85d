"""Config schema and object factories (reference: config_parser/core.py:28-334).

The reference composes YAML with Hydra and validates it with pydantic dataclasses; neither
Hydra nor OmegaConf is installed in this image, so this module carries the same schema
(``GlobalConfig`` with ``train`` / ``datamodule`` / ``model`` / ``analysis`` / ``path`` /
``downstream`` sections, same field names and defaults) plus a small loader that accepts the
reference's YAML files unchanged: ``defaults: [w2v_config]``, ``_target_`` instantiation, and
``key.sub=value`` command-line overrides.

MI355X additions (all optional, defaulted, so reference configs load as they are):
  datamodule.backend      'hip' (device walks straight into the fused kernel) | 'collate'
                          (the reference's DataLoader + W2VCollateFunctional batches)
  datamodule.additional_parameters.rng / seed   walker sampling mode (random_walk_generator)
  train.noise             'torch' (reference-exact CPU noise) | 'device' (Philox on device)
  train.seed              seed for torch / Philox
``_target_: torch.optim.Adam`` instantiates the HIP Adam (word2vec/optim.py, same math).
"""
import copy
import dataclasses
import importlib
import logging
import os
import re
from dataclasses import dataclass, field
from typing import Any, Dict, Iterator, List, Optional, Union

import torch
import yaml
from torch import nn
from torch.optim import Optimizer

from shallow_encoders.common.path import CONFIG_PATH, RUNS_PATH

logger = logging.getLogger('ConfigParser')

# reference `_target_`s whose MI355X-native equivalent is substituted at instantiation
TARGET_SUBSTITUTES = {
    'torch.optim.Adam': 'shallow_encoders.word2vec.optim.Adam',
}


def _locate(path: str):
    module, _, name = path.rpartition('.')
    try:
        return getattr(importlib.import_module(module), name)
    except (ImportError, AttributeError):
        # nested attribute (e.g. pkg.mod.Class.method)
        mod, _, outer = module.rpartition('.')
        return getattr(getattr(importlib.import_module(mod), outer), name)


def instantiate(cfg: Dict[str, Any], **kwargs):
    """Hydra-style ``_target_`` instantiation (recursive on nested ``_target_`` dicts)."""
    cfg = dict(cfg)
    target = cfg.pop('_target_')
    target = TARGET_SUBSTITUTES.get(target, target)
    params = {}
    for k, v in cfg.items():
        params[k] = instantiate(v) if isinstance(v, dict) and '_target_' in v else v
    params.update(kwargs)
    return _locate(target)(**params)


@dataclass
class TrainLossConfig:
    negative_samples: int


@dataclass
class TrainConfig:
    experiment: str
    optimizer: dict
    scheduler: dict
    loss: TrainLossConfig
    max_epochs: int
    accelerator: str
    devices: str
    noise: str = 'torch'
    seed: int = 0

    def instantiate_optimizer(self, params: Iterator[nn.Parameter]) -> Optimizer:
        return instantiate(self.optimizer, params=params)

    def instantiate_scheduler(self, optimizer: Optimizer):
        """Option 1: ``{_target_: ...}`` (stepped per epoch); option 2: PL dict with a nested
        ``scheduler`` plus ``interval`` / ``frequency`` (core.py:55-94)."""
        if '_target_' in self.scheduler:
            return instantiate(self.scheduler, optimizer=optimizer)
        assert 'scheduler' in self.scheduler, 'Missing scheduler object in scheduler configuration.'
        scheduler = copy.deepcopy(self.scheduler)
        scheduler['scheduler'] = instantiate(scheduler['scheduler'], optimizer=optimizer)
        return scheduler


@dataclass
class DatamoduleConfig:
    dataset_name: str
    mode: str
    context_radius: int
    max_length: int
    is_graph: bool
    batch_size: int
    num_workers: int
    min_word_frequency: int = 0
    lemmatize: bool = False
    additional_parameters: dict = field(default_factory=dict)
    backend: str = 'hip'

    def instantiate_dataset(self):
        from shallow_encoders.word2vec.dataloader.torch_dataset import GraphDataset, W2VDataset
        if self.is_graph:
            if self.min_word_frequency > 0:
                logger.warning('Min word frequency has no effect for graph datasets.')
            if self.lemmatize:
                logger.warning('Lemmatization does not have effect on graph datasets.')
            return GraphDataset(dataset_name=self.dataset_name,
                                context_radius=self.context_radius,
                                additional_parameters=self.additional_parameters)
        return W2VDataset(dataset_name=self.dataset_name, context_radius=self.context_radius,
                          min_word_frequency=self.min_word_frequency, lemmatize=self.lemmatize,
                          additional_parameters=self.additional_parameters)

    def instantiate_collate_fn(self):
        from shallow_encoders.word2vec.dataloader.torch_dataset import W2VCollateFunctional
        return W2VCollateFunctional(mode=self.mode, context_radius=self.context_radius,
                                    max_length=self.max_length)

    def instantiate_dataloader(self, dataset=None):
        """backend 'hip' + graph + sg: an iterable of device walk batches; otherwise the
        reference's torch DataLoader with W2VCollateFunctional (num_workers honoured)."""
        dataset = self.instantiate_dataset() if dataset is None else dataset
        if self.backend == 'hip' and self.is_graph and self.mode.lower() == 'sg':
            return WalkBatchLoader(dataset, self.batch_size)
        from torch.utils.data import DataLoader
        return DataLoader(dataset, batch_size=self.batch_size, num_workers=self.num_workers,
                          collate_fn=self.instantiate_collate_fn())


class WalkBatchLoader:
    """Re-iterable epoch source of device walk batches (int32 [batch_size, L])."""

    def __init__(self, dataset, batch_size: int):
        self.dataset = dataset
        self.batch_size = batch_size

    def __iter__(self):
        return iter(self.dataset.walk_batches(self.batch_size))

    def __len__(self) -> int:
        n = len(self.dataset.dataset)
        return (n + self.batch_size - 1) // self.batch_size


@dataclass
class ModelClosestPairAnalysisConfig:
    enable: bool = True
    max_words: int = 100
    pairs_per_word: int = 5


@dataclass
class ModelVisualizeEmbeddingsAnalysisConfig:
    enable: bool = True
    annotate: bool = True
    max_words: int = 1000
    skip_unk: bool = True


@dataclass
class ModelSemanticsTestAnalysisConfig:
    enable: bool = True


@dataclass
class ModelAnalysisConfig:
    checkpoint: str = 'last.ckpt'
    closest_pairs: ModelClosestPairAnalysisConfig = field(
        default_factory=ModelClosestPairAnalysisConfig)
    visualize_embeddings: ModelVisualizeEmbeddingsAnalysisConfig = field(
        default_factory=ModelVisualizeEmbeddingsAnalysisConfig)
    semantics_test: ModelSemanticsTestAnalysisConfig = field(
        default_factory=ModelSemanticsTestAnalysisConfig)


DEFAULT_SPLIT_ALGORITHM = {'_target_': 'shallow_encoders.split.TrainTestRatioSplit',
                           'random_state': 42, 'train_ratio': 0.5, 'stratify': False}


@dataclass
class GraphDownstreamNodeClassificationConfig:
    enable: bool = True
    n_experiments: int = 10
    visualize: bool = True
    split_algorithm: Optional[dict] = None
    classifier_params: Optional[dict] = None

    def instantiate_split_algorithm(self):
        """The configured split (reference: config_parser/core.py:217-232). Without one, the
        reference's intended default (train_ratio 0.5, seed 42, not stratified) is used; the
        reference records that default but then instantiates the missing entry."""
        if self.split_algorithm is None:
            self.split_algorithm = dict(DEFAULT_SPLIT_ALGORITHM)
        return instantiate(self.split_algorithm)


@dataclass
class GraphDownstreamEdgeClassificationConfig:
    enable: bool = True
    operator_name: str = 'hadamard'
    train_ratio: float = 0.5
    n_experiments: int = 10
    classifier_params: Optional[dict] = None


@dataclass
class GraphDownstreamTaskConfig:
    checkpoint: str = 'last.ckpt'
    node_classification: GraphDownstreamNodeClassificationConfig = field(
        default_factory=GraphDownstreamNodeClassificationConfig)
    edge_classification: GraphDownstreamEdgeClassificationConfig = field(
        default_factory=GraphDownstreamEdgeClassificationConfig)


@dataclass
class PathConfig:
    output_dir: str = RUNS_PATH


@dataclass
class GlobalConfig:
    train: TrainConfig
    datamodule: DatamoduleConfig
    model: dict
    analysis: ModelAnalysisConfig = field(default_factory=ModelAnalysisConfig)
    path: PathConfig = field(default_factory=PathConfig)
    downstream: GraphDownstreamTaskConfig = field(default_factory=GraphDownstreamTaskConfig)

    def instantiate_model(self, dataset=None):
        dataset = self.datamodule.instantiate_dataset() if dataset is None else dataset
        return instantiate(self.model, vocab_size=len(dataset.vocab))

    def instantiate_trainer(self, model=None, optimizer=None, scheduler=None, dataset=None,
                            checkpoint_path: Optional[str] = None, device=None):
        from shallow_encoders.word2vec.trainer import Word2VecTrainer
        dataset = self.datamodule.instantiate_dataset() if dataset is None else dataset
        model = self.instantiate_model(dataset=dataset) if model is None else model
        if checkpoint_path is not None:
            state = torch.load(checkpoint_path, map_location='cpu', weights_only=True)
            sd = state.get('state_dict', state)
            sd = {k[len('_model.'):] if k.startswith('_model.') else k: v for k, v in sd.items()}
            model.load_state_dict(sd)
        if device is not None:
            model = model.to(device)
        elif torch.cuda.is_available():
            model = model.cuda()
        optimizer = self.train.instantiate_optimizer(model.parameters()) \
            if optimizer is None else optimizer
        scheduler = self.train.instantiate_scheduler(optimizer) if scheduler is None else scheduler
        return Word2VecTrainer(model=model, optimizer=optimizer, scheduler=scheduler,
                               neg_samples=self.train.loss.negative_samples,
                               vocab_size=len(dataset.vocab), noise=self.train.noise,
                               seed=self.train.seed,
                               context_radius=self.datamodule.context_radius)


# ------------------------------------------------------------------------------- loading
def _from_dict(cls, data):
    if not dataclasses.is_dataclass(cls):
        return data
    if data is None:
        data = {}
    if not isinstance(data, dict):
        raise TypeError(f'{cls.__name__}: expected a mapping, got {type(data).__name__}')
    kwargs = {}
    names = {f.name: f for f in dataclasses.fields(cls)}
    unknown = set(data) - set(names)
    if unknown:
        raise KeyError(f'{cls.__name__}: unknown config keys {sorted(unknown)}')
    for name, f in names.items():
        if name not in data:
            continue
        ftype = f.type if not isinstance(f.type, str) else _resolve_type(f.type)
        kwargs[name] = _from_dict(ftype, data[name]) if dataclasses.is_dataclass(ftype) \
            else data[name]
    return cls(**kwargs)


class _ConfigLoader(yaml.SafeLoader):
    """SafeLoader whose floats follow YAML 1.2 / OmegaConf (the reference's loader): ``1e-3``
    and ``1E+2`` are floats, not strings."""


_ConfigLoader.add_implicit_resolver(
    'tag:yaml.org,2002:float',
    re.compile(r'''^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                |\.[0-9_]+(?:[eE][-+]?[0-9]+)?
                |[-+]?\.(?:inf|Inf|INF)
                |\.(?:nan|NaN|NAN))$''', re.X),
    list('-+0123456789.'))


def _yaml(text_or_stream):
    return yaml.load(text_or_stream, Loader=_ConfigLoader)


def _resolve_type(name: str):
    return globals().get(name, object)


def _parse_value(text: str):
    return _yaml(text)


def apply_overrides(cfg: Dict[str, Any], overrides: List[str]) -> Dict[str, Any]:
    """Apply ``a.b.c=value`` overrides (YAML-typed values) to a nested dict in place."""
    for ov in overrides:
        key, sep, value = ov.partition('=')
        if not sep:
            raise ValueError(f'override "{ov}" is not key=value')
        key = key.lstrip('+')
        node = cfg
        parts = key.split('.')
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = _parse_value(value)
    return cfg


def load_config_dict(config_name: str, config_path: str = CONFIG_PATH,
                     overrides: Optional[List[str]] = None) -> Dict[str, Any]:
    name = config_name if config_name.endswith('.yaml') else config_name + '.yaml'
    path = name if os.path.isabs(name) else os.path.join(config_path, name)
    with open(path, 'r', encoding='utf-8') as f:
        raw = _yaml(f) or {}
    defaults = raw.pop('defaults', [])
    for d in defaults:
        if d not in ('w2v_config', '_self_'):
            raise ValueError(f'unsupported defaults entry {d!r} (only w2v_config)')
    return apply_overrides(raw, list(overrides or []))


def config_from_dict(data: Dict[str, Any]) -> GlobalConfig:
    data = copy.deepcopy(data)
    data.pop('output_dir', None)  # top-level key read by tools/utils.py (reference quirk)
    return _from_dict(GlobalConfig, data)


def load_config(config_name: str, config_path: str = CONFIG_PATH,
                overrides: Optional[List[str]] = None) -> GlobalConfig:
    """Load a reference-style YAML config (``defaults: [w2v_config]``) into GlobalConfig."""
    return config_from_dict(load_config_dict(config_name, config_path, overrides))


def to_yaml(cfg: Union[GlobalConfig, Dict[str, Any]]) -> str:
    data = dataclasses.asdict(cfg) if dataclasses.is_dataclass(cfg) else cfg
    return yaml.safe_dump(data, sort_keys=False)
