"""Optimizer helpers (reference: word2vec/utils/torch_helper.py:7-30)."""
from torch.optim import Optimizer


def get_optim_lr(optimizer: Optimizer) -> float:
    """Learning rate of the first parameter group."""
    for param_group in optimizer.param_groups:
        return param_group['lr']


def set_optim_lr(optimizer: Optimizer, lr: float) -> None:
    """Set the learning rate of every parameter group."""
    for param_group in optimizer.param_groups:
        param_group['lr'] = lr
