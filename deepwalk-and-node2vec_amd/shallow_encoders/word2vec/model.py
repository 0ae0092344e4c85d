"""Word2vec models (reference: word2vec/model.py:10-110).

Same module structure and state_dict keys (``_input_embedding.weight``,
``_output_embedding.weight``) as the reference, so checkpoints and analysis tools interoperate.
On HIP tensors ``SkipGram.forward`` runs the gfx950 logits kernel (and its backward) through
libdw_hip; the training hot path does not call it at all — it runs the fused SGNS kernel
(word2vec/sgns.py), which never materialises logits.
"""
from typing import Optional

import torch
from torch import nn

from shallow_encoders import _native


class W2VBase(nn.Module):
    """Input (centre) and output (context) embedding tables, Xavier-uniform initialised."""

    def __init__(self, vocab_size: int, embedding_size: int, max_norm: Optional[float] = None):
        super().__init__()
        self._input_embedding = nn.Embedding(vocab_size, embedding_size, max_norm=max_norm)
        self._output_embedding = nn.Embedding(vocab_size, embedding_size, max_norm=max_norm)
        torch.nn.init.xavier_uniform_(self._input_embedding.weight)
        torch.nn.init.xavier_uniform_(self._output_embedding.weight)

    @property
    def vocab_size(self) -> int:
        return self._input_embedding.num_embeddings

    @property
    def embedding_size(self) -> int:
        return self._input_embedding.embedding_dim

    @property
    def max_norm(self) -> Optional[float]:
        return self._input_embedding.max_norm

    @property
    def input_embedding(self) -> torch.Tensor:
        """Input embedding weights (CPU copy)."""
        return self._input_embedding.weight.to('cpu').data

    @property
    def output_embedding(self) -> torch.Tensor:
        """Output embedding weights (CPU copy)."""
        return self._output_embedding.weight.to('cpu').data

    @property
    def input_weight(self) -> nn.Parameter:
        return self._input_embedding.weight

    @property
    def output_weight(self) -> nn.Parameter:
        return self._output_embedding.weight

    def embed_inputs(self, inputs: torch.Tensor) -> torch.Tensor:
        return self._input_embedding(inputs)

    def embed_outs(self, outputs: torch.Tensor) -> torch.Tensor:
        return self._output_embedding(outputs)


class _Logits(torch.autograd.Function):
    """logits[b, n] = <mean_p w_in[inputs[b, p]], w_out[outputs[b, n]]> on gfx950
    (SkipGram: P = 1, model.py:85-88; CBOW: P = context width, model.py:104-107)."""

    @staticmethod
    def forward(ctx, w_in, w_out, inputs, outputs):
        B, N = outputs.shape
        P = inputs.shape[1]
        V, d = w_in.shape
        logits = torch.empty((B, N), dtype=torch.float32, device=w_in.device)
        status = torch.zeros(1, dtype=torch.int32, device=w_in.device)
        with torch.cuda.device(w_in.device):
            _native.call('dw_pooled_logits', _native.ptr(inputs), P, _native.ptr(outputs), B, N,
                         V, d, _native.ptr(w_in.detach()), _native.ptr(w_out.detach()), 0,
                         _native.ptr(logits), _native.ptr(status), _native.stream(w_in.device))
        ctx.save_for_backward(w_in, w_out, inputs, outputs, status)
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        w_in, w_out, inputs, outputs, status = ctx.saved_tensors
        B, N = outputs.shape
        P = inputs.shape[1]
        V, d = w_in.shape
        g_in = torch.zeros_like(w_in)
        g_out = torch.zeros_like(w_out)
        with torch.cuda.device(w_in.device):
            _native.call('dw_pooled_logits_backward', _native.ptr(inputs), P,
                         _native.ptr(outputs), B, N, V, d, _native.ptr(w_in.detach()),
                         _native.ptr(w_out.detach()), _native.ptr(dlogits.contiguous().float()),
                         _native.ptr(g_in), _native.ptr(g_out), _native.ptr(status),
                         _native.stream(w_in.device))
        return g_in, g_out, None, None


def _hip_logits(model: 'W2VBase', inputs: torch.Tensor, outputs: torch.Tensor,
                proba: bool) -> torch.Tensor:
    w_in, w_out = model.input_weight, model.output_weight
    if w_in.device.type != 'cuda':
        raise NotImplementedError(
            f'{type(model).__name__}.forward runs on the HIP device only (move the model with '
            '.cuda()); the CPU restatement of the reference lives in oracle/ for tests')
    dev = w_in.device
    B = outputs.shape[0]
    inputs = inputs.to(dev, torch.long).reshape(B, -1).contiguous()
    outputs = outputs.to(dev, torch.long).contiguous()
    if model.max_norm is not None:   # nn.Embedding(max_norm): renormalise looked-up rows first
        from shallow_encoders.word2vec.sgns import renorm_
        renorm_(w_in, inputs, model.max_norm)
        renorm_(w_out, outputs, model.max_norm)
    scalars = _Logits.apply(w_in, w_out, inputs, outputs)
    return torch.sigmoid(scalars) if proba else scalars


class SkipGram(W2VBase):
    """Skip-gram: score every output word against the centre word (model.py:75-91)."""

    def forward(self, inputs: torch.Tensor, outputs: torch.Tensor, proba: bool = True) -> torch.Tensor:
        # inputs: (B, 1) centre ids; outputs: (B, N) context / noise ids
        return _hip_logits(self, inputs.reshape(-1, 1), outputs, proba)


class CBOW(W2VBase):
    """Continuous bag of words (model.py:94-110): the input vector is the MEAN of the input
    rows (inputs (B, N), e.g. the 2R context words in 'cbow' collate mode), scored against
    every output row (outputs (B, M)). With (B, 1) inputs it computes what SkipGram does."""

    def forward(self, inputs: torch.Tensor, outputs: torch.Tensor, proba: bool = True) -> torch.Tensor:
        return _hip_logits(self, inputs, outputs, proba)
