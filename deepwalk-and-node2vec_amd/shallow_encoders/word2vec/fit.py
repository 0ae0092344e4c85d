"""Training loop used by tools/train.py (the reference delegates to PL ``Trainer.fit``,
tools/train.py:60-83, which is not installed in this image).

Semantics kept from PL's automatic optimisation (SURVEY.md §8c "PL loop semantics"):
one ``optimizer.step()`` per batch, gradients zeroed every step, the scheduler stepped once
per epoch (or per step for ``{'scheduler': ..., 'interval': 'step'}`` configs,
config_parser/core.py:55-94), ``on_train_epoch_end`` metric flush, and a
``ModelCheckpoint(save_top_k=-1, save_last=True)`` equivalent (tools/train.py:74-80): one
``checkpoint_epoch=EEEEEE_step=SSSSSSSSS.ckpt`` per epoch plus ``last.ckpt``, each a
torch-loadable dict whose ``state_dict`` keys are ``_model._input_embedding.weight`` /
``_model._output_embedding.weight`` like a Lightning checkpoint of Word2VecTrainer.
Metrics go to ``metrics.csv`` (one row per logged step / epoch) under the TensorBoard
directory layout of tools/conventions.py.
"""
import csv
import os
import shutil
import threading
import time
from typing import Dict, Iterable, Optional

import torch

from shallow_encoders.word2vec.trainer import Word2VecTrainer


def _snapshot(trainer: Word2VecTrainer, epoch: int, global_step: int) -> dict:
    state = {f'_model.{k}': v.detach().cpu() for k, v in trainer.model.state_dict().items()}
    return {'epoch': epoch, 'global_step': global_step, 'state_dict': state,
            'pytorch-lightning_version': None}


def save_checkpoint(path: str, trainer: Word2VecTrainer, epoch: int, global_step: int) -> None:
    torch.save(_snapshot(trainer, epoch, global_step), path)


class _CheckpointWriter:
    """Epoch checkpoints written on a background thread: the tables are copied to the host at
    the epoch boundary (the values of that step), the file writes overlap the next epoch.
    ``last.ckpt`` is a copy of the epoch file, not a second serialisation."""

    def __init__(self, dirpath: str):
        self.dirpath = dirpath
        self._thread = None
        self._error = None

    def _write(self, snap: dict, name: str) -> None:
        try:
            path = os.path.join(self.dirpath, name)
            torch.save(snap, path)
            shutil.copyfile(path, os.path.join(self.dirpath, 'last.ckpt'))
        except BaseException as e:  # re-raised in the training thread by join()
            self._error = e

    def submit(self, trainer: Word2VecTrainer, epoch: int, global_step: int) -> None:
        self.join()
        snap = _snapshot(trainer, epoch, global_step)
        name = f'checkpoint_epoch={epoch:06d}_step={global_step:09d}.ckpt'
        self._thread = threading.Thread(target=self._write, args=(snap, name), daemon=False)
        self._thread.start()

    def join(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None
        if self._error is not None:
            e, self._error = self._error, None
            raise e


class CSVMetricLogger:
    """metrics.csv with columns step, epoch, name, value."""

    def __init__(self, dirpath: Optional[str]):
        self.dirpath = dirpath
        self._rows = []
        if dirpath:
            os.makedirs(dirpath, exist_ok=True)

    def log(self, step: int, epoch: int, values: Dict[str, float]) -> None:
        for k, v in values.items():
            self._rows.append((step, epoch, k, float(v)))

    def flush(self) -> None:
        if not self.dirpath or not self._rows:
            return
        path = os.path.join(self.dirpath, 'metrics.csv')
        new = not os.path.exists(path)
        with open(path, 'a', newline='') as f:
            w = csv.writer(f)
            if new:
                w.writerow(['step', 'epoch', 'name', 'value'])
            w.writerows(self._rows)
        self._rows = []


def _graph_source(trainer: Word2VecTrainer, dataloader, step_sched: bool):
    """The RandomWalkDataset behind a walk-batch loader whose steps can be replayed as HIP graphs
    (word2vec/graphed.py GraphedTrainerStep), or None. DW_TRAIN_GRAPH=0 keeps every step eager;
    DW_TRAIN_GRAPH_SCATTER=records makes the graphs take the eager loop's records step even
    where the atomic scatter is faster (GraphedTrainerStep's ``scatter``)."""
    from shallow_encoders.config_parser.core import WalkBatchLoader
    from shallow_encoders.word2vec.graphed import GraphedTrainerStep
    if os.environ.get('DW_TRAIN_GRAPH', '1') == '0' or step_sched:
        return None
    if not isinstance(dataloader, WalkBatchLoader) or not torch.cuda.is_available():
        return None
    rwd = dataloader.dataset.dataset
    R = trainer._context_radius
    if R is None or rwd.walk_length < 2 * R + 1:
        return None
    return rwd if GraphedTrainerStep.eligible(trainer, rwd) else None


def fit(trainer: Word2VecTrainer, dataloader: Iterable, max_epochs: int,
        checkpoint_dir: Optional[str] = None, log_dir: Optional[str] = None,
        log_every_n_steps: int = 50, verbose: bool = True,
        graph_unroll: int = 16) -> Dict[str, float]:
    """Train for ``max_epochs``; returns the last epoch's metric means.

    Device walk batches (Philox walks or the reference's own, rng='python'; device or torch
    negatives) are replayed ``graph_unroll`` steps per HIP graph after each epoch's first (eager)
    batch
    (GraphedTrainerStep), without a Python launch per kernel. The trailing batches that do not
    fill a graph, and everything else, run eagerly. The replayed steps train the same batches with
    the same update, but with DW_TRAIN_GRAPH_SCATTER='auto' (the default) a batch of at most
    65,536 output records (the reference configs' 64-walk batches) takes the atomic output-table
    scatter and one Adam launch over both tables, where the eager step sorts the records and
    fuses the out table's Adam into their gather: the same sums in another float order, so the
    tables agree to float-atomic rounding, not bit for bit. 'records' replays the eager step's
    own kernels."""
    from shallow_encoders.word2vec.graphed import GraphedTrainerStep
    trainer.manual_grads = True
    opt = trainer.optimizer
    sched = trainer.scheduler
    step_sched = isinstance(sched, dict) and sched.get('interval', 'epoch') == 'step'
    sched_obj = sched['scheduler'] if isinstance(sched, dict) else sched
    logger = CSVMetricLogger(log_dir)
    writer = None
    if checkpoint_dir:
        os.makedirs(checkpoint_dir, exist_ok=True)
        writer = _CheckpointWriter(checkpoint_dir)
    global_step = 0
    last = {}
    for epoch in range(max_epochs):
        t0 = time.perf_counter()
        n_batches = 0

        def run(batch):
            nonlocal global_step, n_batches
            loss = trainer.training_step(batch)
            opt.step()
            opt.zero_grad()
            if step_sched and sched_obj is not None:
                sched_obj.step()
            if log_dir and global_step % log_every_n_steps == 0:
                logger.log(global_step, epoch, {f'train/{k}': v for k, v in loss.items()})
            global_step += 1
            n_batches += 1

        rwd = _graph_source(trainer, dataloader, step_sched)
        if rwd is None:
            for batch in dataloader:
                run(batch)
        else:
            B = dataloader.batch_size
            batch = rwd.next_walk_batch(B, check=False)   # eager: creates state / workspaces
            if batch is not None:
                run(batch)
                n_rep = (len(rwd) - rwd._index) // B // graph_unroll
                if n_rep > 0:
                    gs = GraphedTrainerStep(trainer, rwd, B, n_rep * graph_unroll, graph_unroll,
                                            os.environ.get('DW_TRAIN_GRAPH_SCATTER', 'auto'))
                    for _ in range(n_rep):
                        loss = trainer.push_replayed(gs.replay(), graph_unroll)
                        if log_dir and (-global_step) % log_every_n_steps < graph_unroll:
                            logger.log(global_step + (-global_step) % log_every_n_steps, epoch,
                                       {f'train/{k}': v for k, v in loss.items()})
                        global_step += graph_unroll
                        n_batches += graph_unroll
                    torch.cuda.current_stream().synchronize()
                    gs.release_rng()   # the reference's streams back to random / torch
                    from shallow_encoders import _native
                    _native.check_status(gs.status, 'graphed training steps')
                while True:
                    batch = rwd.next_walk_batch(B, check=False)
                    if batch is None:
                        break
                    run(batch)
        last = trainer.on_train_epoch_end()         # synchronises with the device
        t_loop = time.perf_counter() - t0
        if not step_sched and sched_obj is not None:
            sched_obj.step()
        last['epoch/lr'] = float(opt.param_groups[0]['lr'])
        logger.log(global_step, epoch, last)
        logger.flush()
        if writer is not None:
            writer.submit(trainer, epoch, global_step)
        if verbose:
            dt = time.perf_counter() - t0
            msg = ' '.join(f'{k}={v:.4f}' for k, v in last.items() if k.endswith('loss'))
            print(f'epoch {epoch}: {n_batches} batches in {dt:.2f}s (training loop {t_loop:.2f}s) '
                  f'{msg}', flush=True)
    if writer is not None:
        writer.join()
    return last
