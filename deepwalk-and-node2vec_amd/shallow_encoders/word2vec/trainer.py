"""Word2VecTrainer (reference: word2vec/trainer.py:18-165) on the fused gfx950 SGNS kernel.

Keeps the reference surface — ``Word2VecTrainer(model, optimizer, scheduler, neg_samples,
vocab_size)``, ``.model/.optimizer/.scheduler``, ``training_step(batch) -> loss dict``,
``on_train_epoch_end``, ``configure_optimizers() -> ([opt], [sched])`` and the logged metric
names (``train/loss``, ``train/positive-loss``, ``train/negative-loss``, ``epoch/lr``,
``train-epoch/*``, ``train-metrics/recall``, ``train-metrics/precision``).

``training_step`` accepts either batch format:
  * ``(inputs, targets)`` from W2VCollateFunctional (the reference's format), or
  * a device int32 walk tensor [n_walks, L] (GraphDataset.walk_batches): windows are formed
    inside the kernel, nothing is materialised on the host.

Gradient delivery:
  * ``manual_grads = True`` (the in-repo loop, tools/train.py, bench.py): the kernel adds the
    gradient of the batch-mean loss straight into ``param.grad``; the HIP Adam step consumes
    and zeroes it. No autograd graph, no host synchronisation per step.
  * ``manual_grads = False`` (default; a Lightning-style loop calling ``loss.backward()``):
    the returned ``loss`` carries a grad_fn whose backward hands over the same gradients.

Fused step (``manual_grads`` + walk batches + the HIP Adam holding exactly the two tables, one
device, records path): ``training_step`` also applies the optimizer update, the way bench.py's
step does. The three pieces run as follows:
  * SGNS pass 1 runs first, after which the input-table gradient is final.
  * The input table's Adam then runs on a side stream, out of place into the table's second
    buffer, overlapping the output-table phase, which still reads the current input table.
  * The output table's Adam is fused into that phase's records gather
    (dw_sgns_walks_phase2_adam).
The optimizer's ``step()`` that follows is then a no-op for the two tables (Adam.begin_fused_step).
Same update as SGNS + ``optimizer.step()`` up to float-atomic summation order
(test_gpu_trainer.py::test_fused_trainer_step_equals_unfused).

Noise: ``noise='torch'`` draws the reference's uniform negatives with torch's global CPU
generator (generate_noise_batch, exact under ``torch.manual_seed``); ``noise='device'`` draws
the same law on the device (Philox keyed by ``seed`` and the running centre counter).

Deviation (documented): per-step loss values stay on the device; the reference's per-step
``.detach().cpu()`` NaN assert (trainer.py:116,121) runs once per epoch instead.
"""
from typing import Dict, List, Union

import torch
from torch.optim import Optimizer

from shallow_encoders import _native
from shallow_encoders.word2vec import exact
from shallow_encoders.word2vec.model import W2VBase
from shallow_encoders.word2vec.sgns import (SGNSLoss, _use_records, device_noise, loss_terms,
                                            renorm_, sgns_accumulate, sgns_phase_bytes)
from shallow_encoders.word2vec.utils import torch_helper
from shallow_encoders.word2vec.utils.meter import MetricMeter
from shallow_encoders.word2vec.utils.sampling import generate_noise_batch

try:  # keep Lightning compatibility when it is installed (it is not in this image)
    import pytorch_lightning as _pl
    _Base = _pl.LightningModule
    _HAS_PL = True
except ImportError:  # pragma: no cover - depends on the environment
    _Base = torch.nn.Module
    _HAS_PL = False


class Word2VecTrainer(_Base):
    """Trains a W2V model with the fused SGNS kernel."""

    def __init__(self, model: W2VBase, optimizer: Optimizer, scheduler, neg_samples: int,
                 vocab_size: int, noise: str = 'torch', seed: int = 0, context_radius: int = None):
        super().__init__()
        if noise not in ('torch', 'device'):
            raise ValueError('noise must be "torch" or "device"')
        self._optimizer = optimizer
        self._scheduler = scheduler
        self._neg_samples = neg_samples
        self._vocab_size = vocab_size
        self._model = model
        self._meter = MetricMeter()
        self._noise_mode = noise
        self._seed = int(seed)
        self._noise_offset = 0
        self._context_radius = context_radius
        self.manual_grads = False
        self.logged: Dict[str, object] = {}
        self._side = None          # side stream of the fused step (input-table Adam)
        self._row_flags = None     # fused output-table Adam scratch
        # set while word2vec/graphed.py GraphedTrainerStep captures the step: the steps add
        # their loss sums here and skip the per-step metrics (read once per replay), and
        # _capture_scatter = 'atomic' takes the atomic output-table scatter (tiny batches)
        self._capture_acc = None
        self._capture_scatter = None
        # set by GraphedTrainerStep for noise='torch': the step's negatives, already drawn on the
        # device from torch's generator stream (graph/rng.py DeviceMT.randint)
        self._noise_override = None
        # the deterministic mode's accumulators (word2vec/exact.py; DW_DETERMINISTIC=1)
        self._exact = None

    # ---- reference properties -------------------------------------------------------------
    @property
    def model(self) -> W2VBase:
        return self._model

    @property
    def optimizer(self) -> Optimizer:
        return self._optimizer

    @optimizer.setter
    def optimizer(self, optimizer: Optimizer) -> None:
        self._optimizer = optimizer

    @property
    def scheduler(self):
        return self._scheduler

    @scheduler.setter
    def scheduler(self, scheduler) -> None:
        self._scheduler = scheduler

    @property
    def meter(self) -> MetricMeter:
        return self._meter

    # ---- logging ------------------------------------------------------------------------------
    def log(self, name: str, value, prog_bar: bool = False, **kwargs) -> None:  # noqa: D401
        if _HAS_PL and getattr(self, '_trainer', None) is not None:
            return super().log(name, value, prog_bar=prog_bar, **kwargs)
        self.logged[name] = value
        return None

    def _log_loss(self, loss: Dict[str, torch.Tensor], prefix: str, log_step: bool = True) -> None:
        assert prefix in ['train', 'val'], f'Invalid prefix value "{prefix}"!'
        assert 'loss' in loss, \
            f'When returning loss as dictionary it has to have key "loss". Found: {list(loss.keys())}'
        for name, value in loss.items():
            value = value.detach()
            self._meter.push(f'{prefix}-epoch/{name}', value)
            if log_step:
                self.log(f'{prefix}/{name}', value, prog_bar=False)

    def forward(self, inputs: torch.Tensor, outputs: torch.Tensor, proba: bool = True) -> torch.Tensor:
        return self._model(inputs, outputs, proba=proba)

    # ---- training -----------------------------------------------------------------------------
    def _status(self, device) -> torch.Tensor:
        st = getattr(self, '_renorm_status', None)
        if st is None or st.device != device:
            st = torch.zeros(1, dtype=torch.int32, device=device)
            self._renorm_status = st
        return st

    def _noise(self, n_centres: int, n_ctx: int, device) -> Union[torch.Tensor, None]:
        if self._noise_mode == 'device':
            return None
        if self._noise_override is not None:
            return self._noise_override
        noise = generate_noise_batch(n_centres, n_ctx, self._neg_samples, self._vocab_size)
        return noise.to(device, non_blocking=True)

    def training_step(self, batch, *args, **kwargs) -> Dict[str, torch.Tensor]:
        w_in = self._model.input_weight
        w_out = self._model.output_weight
        dev = w_in.device
        if isinstance(batch, torch.Tensor):           # device walks [n, L]
            R = self._context_radius
            if R is None:
                raise ValueError('walk batches need context_radius (set it on the trainer)')
            walks = batch if batch.dtype == torch.int32 else batch.to(torch.int32)
            walks = walks.to(dev).contiguous()
            n, L = walks.shape
            n_centres, C = n * (L - 2 * R), 2 * R
            src, targets = walks, None
        else:                                         # (inputs, targets) from the collate fn
            inputs, targets = batch                   # sg: (B, 1), (B, 2R); cbow: (B, 2R), (B, 1)
            targets = targets.to(dev, torch.long).contiguous()
            n_centres, C = targets.shape
            src = inputs.to(dev, torch.long).reshape(n_centres, -1).contiguous()
            if src.shape[1] == 1:
                src = src.reshape(-1)
            R = C // 2
        noise = self._noise(n_centres, C, dev)
        offset = self._noise_offset
        self._noise_offset += n_centres
        max_norm = self._model.max_norm
        if max_norm is not None:
            # nn.Embedding(max_norm) renormalises every row the reference's two forwards look
            # up (inputs in the in table; targets and negatives in the out table) before the
            # loss: materialise the device negatives, renormalise, then run the fused step
            if targets is None:
                raise NotImplementedError('max_norm with device walk batches: use the collate '
                                          '(pairs) dataloader')
            if noise is None:
                noise = device_noise(n_centres, C, self._neg_samples, self._vocab_size,
                                     self._seed, offset, dev)
            st = self._status(dev)
            renorm_(w_in, src, max_norm, st)
            renorm_(w_out, targets, max_norm, st)
            renorm_(w_out, noise, max_norm, st)
        if self.manual_grads:
            from shallow_encoders.word2vec.optim import Adam
            fresh = [p for p in (w_in, w_out) if p.grad is None]
            for p in fresh:
                p.grad = torch.zeros_like(p)
            if isinstance(self._optimizer, Adam):
                self._optimizer.mark_grads(fresh, True)
            if exact.enabled():   # int64 fixed-point accumulators for the two gradient buffers
                if self._exact is None:
                    self._exact = exact.Registry()
                scale = 1.0 / max(n_centres * C, 1)
                self._exact.ensure(0, w_in.grad, scale)
                self._exact.ensure(1, w_out.grad, scale)
            elif self._exact is not None:
                self._exact.release()
                self._exact = None
            if targets is None and self._capture_scatter != 'atomic' and \
                    self._can_fuse_step(w_in, w_out, C):
                acc = self._fused_walk_step(w_in, w_out, src, R, noise, offset)
            elif targets is None:
                acc = sgns_accumulate(w_in.detach(), w_out.detach(), w_in.grad, w_out.grad,
                                      self._neg_samples, walks=src, context_radius=R, noise=noise,
                                      seed=self._seed, noise_offset=offset,
                                      loss_acc=self._capture_acc,
                                      scatter=self._capture_scatter or 'sorted')
            else:
                acc = sgns_accumulate(w_in.detach(), w_out.detach(), w_in.grad, w_out.grad,
                                      self._neg_samples, inputs=src, targets=targets, noise=noise,
                                      seed=self._seed, noise_offset=offset)
            if isinstance(self._optimizer, Adam) and not self._optimizer._fused_done:
                self._optimizer.mark_grads([w_in, w_out], False)   # accumulated, not consumed
            if self._capture_acc is not None:   # a captured step: metrics once per replay
                return None
            t = loss_terms(acc, n_centres * C, self._neg_samples)
            loss = {k: t[k] for k in ('loss', 'positive-loss', 'negative-loss')}
            recall, precision = t['recall'], t['precision']
        else:
            outs = SGNSLoss.apply(w_in, w_out, src, targets, noise, R, self._neg_samples,
                                  self._seed, offset)
            loss = {'loss': outs[0], 'positive-loss': outs[1], 'negative-loss': outs[2]}
            recall, precision = outs[3], outs[4]
        self._log_loss(loss, prefix='train', log_step=True)
        self.log('epoch/lr', torch_helper.get_optim_lr(self.optimizer))
        self._meter.push('train-metrics/recall', recall)
        self._meter.push('train-metrics/precision', precision)
        return loss

    # ---- fused step -----------------------------------------------------------------------------
    def _can_fuse_step(self, w_in, w_out, n_ctx: int) -> bool:
        from shallow_encoders.word2vec.optim import Adam
        opt = self._optimizer
        return (isinstance(opt, Adam) and w_in.device.type == 'cuda'
                and _use_records('sorted', n_ctx, self._neg_samples, w_in.shape[0])
                and opt.can_fuse([w_in, w_out]))

    def _fused_walk_step(self, w_in, w_out, walks, R: int, noise, offset: int) -> torch.Tensor:
        """Pass 1 -> input-table Adam on the side stream (into the second buffer) || output-table
        phase with its Adam fused -> join -> swap the input table's buffers."""
        from shallow_encoders.word2vec.sharding import adam_to_scalars, overlap_adam_blocks
        opt = self._optimizer
        (st_in, sc_in), (st_out, sc_out) = opt.begin_fused_step([w_in, w_out])
        dev = w_in.device
        K = self._neg_samples
        V, d = w_in.shape
        n, L = walks.shape
        kw = dict(walks=walks, context_radius=R, noise=noise, seed=self._seed,
                  noise_offset=offset)
        acc = sgns_accumulate(w_in.detach(), w_out.detach(), w_in.grad, w_out.grad, K,
                              phase=1, loss_acc=self._capture_acc, **kw)
        if self._side is None or self._side.device != dev:
            self._side = torch.cuda.Stream(dev)
        if self._row_flags is None or self._row_flags.numel() != V or \
                self._row_flags.device != dev:
            self._row_flags = torch.zeros(V, dtype=torch.uint8, device=dev)
        alt = opt.alt_buffer(w_in)
        main = torch.cuda.current_stream(dev)
        ready = torch.cuda.Event()
        ready.record(main)
        pb = sgns_phase_bytes(n, L, R, K, d, V, 'sorted', True)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            adam_to_scalars(w_in.detach(), alt, w_in.grad, st_in['exp_avg'],
                            st_in['exp_avg_sq'], sc_in, True,
                            overlap_adam_blocks(V * d * 4 * 7, pb['sort'] + pb['pass2']))
            done = torch.cuda.Event()
            done.record(self._side)
        sgns_accumulate(w_in.detach(), w_out.detach(), w_in.grad, w_out.grad, K, phase=2,
                        loss_acc=acc,
                        out_adam={'m': st_out['exp_avg'], 'v': st_out['exp_avg_sq'],
                                  'flags': self._row_flags, 'scalars': sc_out}, **kw)
        main.wait_event(done)
        opt.swap_alt(w_in)
        return acc

    def push_replayed(self, terms: Dict[str, torch.Tensor], n_steps: int) -> Dict[str, torch.Tensor]:
        """The metrics of ``n_steps`` graph-replayed steps (word2vec/graphed.py
        GraphedTrainerStep): their mean loss terms stand for each of the steps in the epoch
        means, as training_step's per-step pushes would; returns the loss dict."""
        loss = {k: terms[k] for k in ('loss', 'positive-loss', 'negative-loss')}
        for _ in range(n_steps):
            self._log_loss(loss, prefix='train', log_step=False)
            self._meter.push('train-metrics/recall', terms['recall'])
            self._meter.push('train-metrics/precision', terms['precision'])
        for name, value in loss.items():
            self.log(f'train/{name}', value)
        self.log('epoch/lr', torch_helper.get_optim_lr(self.optimizer))
        return loss

    def on_train_epoch_end(self) -> Dict[str, float]:
        """Log the epoch means; one host synchronisation per epoch (NaN check included)."""
        st = getattr(self, '_renorm_status', None)
        if st is not None:
            _native.check_status(st, 'max_norm renormalisation')
        if self._meter.is_empty:
            return {}
        out = {}
        for name, value in self._meter.get_all():
            v = float(value)
            assert v == v, f'Got nan value for key "{name}"!'
            out[name] = v
            self.log(name, v, prog_bar=name.endswith('/loss'))
        return out

    def configure_optimizers(self):
        return [self._optimizer], [self._scheduler]
