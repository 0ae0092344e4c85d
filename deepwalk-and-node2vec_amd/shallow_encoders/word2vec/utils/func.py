"""Tensor helpers (reference: word2vec/utils/func.py)."""
import torch


def pairwise_cosine_similarity(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """cos(x_i, y_j) for every row pair: [n, d] x [m, d] -> [n, m] (rows normalised by their
    L2 norm, then one matrix product)."""
    x = x / torch.norm(x, dim=-1, keepdim=True)
    y = y / torch.norm(y, dim=-1, keepdim=True)
    return x @ y.T
