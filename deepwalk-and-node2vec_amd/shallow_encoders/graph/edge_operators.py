"""Edge embeddings from node embeddings: vector(edge(n1, n2)) = f(vector(n1), vector(n2)).

Reference: shallow_encoders/graph/edge_operators.py (average, hadamard, weighted_l1,
weighted_l2 and ``edge_operator_factory``). Each operator works on single vectors and on
row-stacked batches alike (numpy broadcasting), so the downstream tool builds all edge
embeddings of an experiment in one call instead of a Python loop per edge.
"""
from typing import Callable

import numpy as np


def average(lhs: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    """(n1 + n2) / 2."""
    return (lhs + rhs) / 2


def hadamard(lhs: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    """Element-wise product n1 * n2."""
    return lhs * rhs


def weighted_l1(lhs: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    """Element-wise |n1 - n2|."""
    return np.abs(lhs - rhs)


def weighted_l2(lhs: np.ndarray, rhs: np.ndarray) -> np.ndarray:
    """Element-wise (n1 - n2)^2."""
    return (lhs - rhs) ** 2


EdgeOperator = Callable[[np.ndarray, np.ndarray], np.ndarray]

EDGE_OPERATORS = {
    'average': average,
    'hadamard': hadamard,
    'weighted_l1': weighted_l1,
    'weighted_l2': weighted_l2,
}


def edge_operator_factory(name: str) -> EdgeOperator:
    """Operator by (case-insensitive) name; unknown names raise AssertionError like the
    reference."""
    name = name.lower()
    assert name in EDGE_OPERATORS, \
        f'Operator "{name}" is not supported. Available: {list(EDGE_OPERATORS.keys())}'
    return EDGE_OPERATORS[name]


def edge_embeddings(node_embeddings: np.ndarray, edges: np.ndarray,
                    operator: EdgeOperator) -> np.ndarray:
    """Embeddings of edges given as an int array [n, 2] of node indices (row-stacked)."""
    edges = np.asarray(edges, dtype=np.int64).reshape(-1, 2)
    return operator(node_embeddings[edges[:, 0]], node_embeddings[edges[:, 1]])
