"""Negative sampling (reference: word2vec/utils/sampling.py:7-21).

Uniform over [0, vocab_size) — including the ``<unk>`` row and possibly the positive itself —
despite the reference docstring's "uni-gram". Drawn on the host with torch's global CPU
generator, so ``torch.manual_seed`` reproduces the reference's noise exactly; the fused kernel
can instead draw the same law on the device (Philox, ``noise='device'``).
"""
import torch


def generate_noise_batch(batch_size: int, n_words: int, neg_samples: int, vocab_size: int):
    """Noise word ids, shape (batch_size, n_words, neg_samples), int64, CPU."""
    return torch.randint(low=0, high=vocab_size, size=(batch_size, n_words, neg_samples),
                         dtype=torch.long)
