"""Graph random-walk datasets (reference: shallow_encoders/graph/datasets.py:17-221).

``RandomWalkDataset`` keeps the reference's iteration semantics exactly:
  * start-node order ``list(graph)`` shuffled ONCE with the global ``random`` in the
    constructor (datasets.py:42,45), reshuffled at every ``StopIteration`` (:86-88);
  * walk index i starts at ``_nodes[i // walks_per_node]`` (:69-76); ``len = N * W`` (:78-79).
``__next__`` still yields one walk string. The batched device API (``next_walk_batch``)
continues the SAME iteration state and, in rng='python' mode, consumes the global ``random``
stream exactly as the same number of ``__next__`` calls would.
"""
import os
from typing import Dict, Optional

import numpy as np
import torch

from shallow_encoders import _native

from shallow_encoders.common.path import ASSETS_PATH
from shallow_encoders.graph.csr import CSRGraph
from shallow_encoders.graph.random_walk_generator import RandomWalk, random_walk_factory
from shallow_encoders.graph.rng import shuffled_range
from shallow_encoders.word2vec.dataloader.registry import register_dataset


class RandomWalkDataset:
    """RandomWalk dataset: a graph (structure) plus a random-walk generator."""

    def __init__(
        self,
        graph,
        walks_per_node: int,
        walk_length: int,
        method: str = 'deepwalk',
        method_params: Optional[dict] = None,
        labels: Optional[Dict[str, str]] = None,
        features: Optional[Dict[str, np.ndarray]] = None,
        rng: str = 'python',
        seed: int = 0,
        device=None,
    ):
        """
        Args:
            graph: networkx Graph (or CSRGraph for synthetic graphs)
            walks_per_node: number of walks generated from each node per epoch
            walk_length: random walk length
            method: 'deepwalk' | 'dfs' | 'node2vec'
            method_params: walker parameters (p, q)
            labels / features: optional node annotations
            rng / seed / device: walker sampling mode (see random_walk_generator)
        """
        self._graph = graph
        if isinstance(graph, CSRGraph):
            base_nodes = list(graph.names[1:])
        else:
            base_nodes = list(graph)
        self._labels = labels
        self._features = features
        # the reference shuffles the node list in place; shuffling an index permutation with
        # the same generator consumes the same draws and yields the same order (native loop)
        self._base_nodes = base_nodes
        self._perm = shuffled_range(len(base_nodes))   # epoch order, as base_nodes indices

        method_params = {} if method_params is None else method_params
        self._walk_generator: RandomWalk = random_walk_factory(
            name=method,
            graph=graph,
            length=walk_length,
            additional_params=method_params,
            rng=rng,
            seed=seed,
            device=device,
        )
        csr = self._walk_generator.csr
        self._base_ids = np.asarray([csr.node_id(n) for n in base_nodes], dtype=np.int32) \
            if not isinstance(graph, CSRGraph) else np.arange(1, len(base_nodes) + 1,
                                                              dtype=np.int32)
        self._node_ids = self._base_ids[self._perm]
        self._walks_per_node = walks_per_node
        self._index = 0
        self._epoch = 0

    # ---- reference surface -------------------------------------------------------------
    @property
    def graph(self):
        return self._graph

    @property
    def walk_generator(self) -> RandomWalk:
        return self._walk_generator

    @property
    def csr(self) -> CSRGraph:
        return self._walk_generator.csr

    @property
    def walks_per_node(self) -> int:
        return self._walks_per_node

    @property
    def walk_length(self) -> int:
        return self._walk_generator.length

    def _get_current_node(self):
        return self._base_nodes[self._perm[self._index // self._walks_per_node]]

    def __len__(self) -> int:
        return len(self._base_nodes) * self._walks_per_node

    def __iter__(self) -> 'RandomWalkDataset':
        self._index = 0
        return self

    def _reshuffle(self) -> None:
        # the reference re-shuffles its node list in place (same draws as shuffling indices);
        # names are looked up through the permutation instead of rebuilding a list of them
        p = shuffled_range(len(self._base_nodes))
        self._perm = self._perm[p]
        self._node_ids = self._node_ids[p]
        self._dev_starts = None
        self._epoch += 1

    def __next__(self):
        if self._index >= len(self):
            self._reshuffle()
            raise StopIteration('Finished.')
        node = self._get_current_node()
        walk = self._walk_generator.walk(node)
        self._index += 1
        return walk

    # ---- batched device API ----------------------------------------------------------------
    def start_ids(self, first: int, count: int) -> np.ndarray:
        """Vocabulary ids of the start nodes of walks [first, first+count) of this epoch."""
        idx = np.arange(first, first + count, dtype=np.int64) // self._walks_per_node
        return self._node_ids[idx]

    def _device_starts(self) -> Optional[torch.Tensor]:
        """The epoch's start ids (int32, one per walk) on the walker's device, copied once per
        epoch, so that a batch needs no host-to-device copy: a copy from pageable host memory
        waits for the stream to drain, which would stall the training pipeline every batch."""
        if not torch.cuda.is_available():
            return None
        dev = _native.require_device(self._walk_generator._device)
        st = getattr(self, '_dev_starts', None)
        if st is None or st.device != dev:
            ids = torch.from_numpy(self._node_ids.astype(np.int32))
            st = ids.to(dev).repeat_interleave(self._walks_per_node)
            self._dev_starts = st
        return st

    def next_walk_batch(self, max_walks: int, check: bool = True) -> Optional[torch.Tensor]:
        """The next <= max_walks walks of the epoch as device int32 [n, L]; None at epoch end
        (which reshuffles, as ``StopIteration`` does, and rewinds like ``__iter__``)."""
        if self._index >= len(self):
            self._reshuffle()
            self._index = 0
            return None
        n = min(int(max_walks), len(self) - self._index)
        starts = self._device_starts()
        if starts is not None:          # a slice of the epoch's start ids, already on the device
            starts = starts[self._index:self._index + n]
        else:
            starts = torch.from_numpy(self.start_ids(self._index, n))
        walk_id0 = self._epoch * len(self) + self._index
        out = self._walk_generator.walk_batch(starts, walk_id0=walk_id0, check=check)
        self._index += n
        return out

    @property
    def has_labels(self) -> bool:
        return self._labels is not None

    @property
    def labels(self) -> Dict[str, str]:
        assert self.has_labels, 'This dataset does not have any labels!'
        return self._labels

    @property
    def has_features(self) -> bool:
        return self._features is not None

    @property
    def features(self) -> Dict[str, np.ndarray]:
        assert self.has_features, 'This dataset does not have any features!'
        return self._features


@register_dataset('graph_triplets')
class GraphTriplets(RandomWalkDataset):
    """NUM_CLUSTERS disjoint 3-node paths x1-x2-x3 (datasets.py:126-151), a sanity dataset."""
    NUM_CLUSTERS = 3

    def __init__(self, walks_per_node: int, walk_length: int, method: str = 'deepwalk', *,
                 rng: str = 'python', seed: int = 0, device=None):
        import networkx as nx
        graph = nx.Graph()
        labels = {}
        for i in range(self.NUM_CLUSTERS):
            prefix = chr(ord('a') + i)
            graph.add_edge(f'{prefix}1', f'{prefix}2')
            graph.add_edge(f'{prefix}2', f'{prefix}3')
            for suffix in ['1', '2', '3']:
                labels[f'{prefix}{suffix}'] = str(i)
        super().__init__(graph=graph, walks_per_node=walks_per_node, walk_length=walk_length,
                         method=method, labels=labels, rng=rng, seed=seed, device=device)


@register_dataset('graph_karate_club')
class KarateClubDataset(RandomWalkDataset):
    """Zachary's karate club, nodes relabelled n01..n34 (datasets.py:154-180)."""

    def __init__(self, walks_per_node: int, walk_length: int, method: str = 'deepwalk',
                 **kwargs):
        import networkx as nx
        graph = nx.karate_club_graph()
        mapping = {node: f'n{node + 1:02d}' for node in graph.nodes}
        graph = nx.relabel_nodes(graph, mapping)
        club = {n: graph.nodes[n].get('club') for n in graph.nodes}
        # community labels of the reference's table (Mr. Hi -> '1', Officer -> '2'); they
        # coincide with networkx's 'club' node attribute
        labels = {n: ('1' if club[n] == 'Mr. Hi' else '2') for n in graph.nodes}
        super().__init__(graph=graph, walks_per_node=walks_per_node, walk_length=walk_length,
                         method=method, labels=labels, **kwargs)


@register_dataset('graph_cora')
class CoraDataset(RandomWalkDataset):
    """Cora citation graph from assets/cora/cora.{cites,content} (datasets.py:183-221).

    The files are not shipped (the reference downloads them, tools/download_dataset.sh);
    without them construction raises FileNotFoundError.
    """

    def __init__(self, walks_per_node: int, walk_length: int, method: str = 'deepwalk',
                 **kwargs):
        import networkx as nx
        import pandas as pd
        cora_dirpath = os.path.join(ASSETS_PATH, 'cora')
        edges_path = os.path.join(cora_dirpath, 'cora.cites')
        nodes_path = os.path.join(cora_dirpath, 'cora.content')
        if not (os.path.exists(edges_path) and os.path.exists(nodes_path)):
            raise FileNotFoundError(f'Cora data not found under {cora_dirpath} '
                                    '(cora.cites, cora.content)')
        edge_list = pd.read_csv(edges_path, sep='\t', header=None, names=['target', 'source'])
        edge_list = edge_list.astype('str')
        edge_list.target = 'n' + edge_list.target
        edge_list.source = 'n' + edge_list.source
        edge_list['label'] = 'cites'
        graph = nx.from_pandas_edgelist(edge_list, edge_attr='label')
        feature_names = [f'w_{ii}' for ii in range(1433)]
        node_data = pd.read_csv(nodes_path, sep='\t', header=None,
                                names=feature_names + ['subject'])
        node_data.index = 'n' + node_data.index.astype(str)
        labels = node_data.subject.to_dict()
        features = {k: np.array(v) for k, v in node_data[feature_names].T.to_dict('list').items()}
        super().__init__(graph=graph, walks_per_node=walks_per_node, walk_length=walk_length,
                         method=method, labels=labels, features=features, **kwargs)


@register_dataset('graph_rmat')
class RMATDataset(RandomWalkDataset):
    """Synthetic R-MAT power-law graph (BASELINE configs C3-C5; spec in graph/rmat.py).

    Built straight to CSR (no networkx): scale 20 / 10M edges is the 1M-node benchmark graph.
    """

    def __init__(self, walks_per_node: int, walk_length: int, method: str = 'deepwalk',
                 scale: int = 20, n_edges: int = 10_000_000, graph_seed: int = 0, **kwargs):
        from shallow_encoders.graph.rmat import rmat_graph
        graph = rmat_graph(scale, n_edges, graph_seed)
        super().__init__(graph=graph, walks_per_node=walks_per_node, walk_length=walk_length,
                         method=method, **kwargs)
