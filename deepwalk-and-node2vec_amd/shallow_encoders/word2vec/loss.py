"""Negative-sampling loss (reference: word2vec/loss.py:14-22).

The training hot path never materialises logits: the fused kernel (word2vec/sgns.py) computes
this loss and its gradient in one pass. This module keeps the reference's loss object for the
unfused API (SkipGram.forward logits -> loss -> autograd).
"""
from typing import Dict

import torch
from torch import nn


class NegativeSamplingLoss(nn.Module):
    """-log clamp(sigmoid(pos), 1e-6) - sum_k log clamp(sigmoid(-neg_k), 1e-6), batch mean."""

    def forward(self, positive_logits: torch.Tensor,
                negative_logits: torch.Tensor) -> Dict[str, torch.Tensor]:
        positive_loss = -torch.log(torch.clamp(torch.sigmoid(positive_logits), min=1e-6))
        negative_loss = -torch.log(torch.clamp(torch.sigmoid(-negative_logits), min=1e-6)).sum(-1)
        return {
            'loss': torch.mean(positive_loss + negative_loss),
            'positive-loss': torch.mean(positive_loss),
            'negative-loss': torch.mean(negative_loss),
        }
