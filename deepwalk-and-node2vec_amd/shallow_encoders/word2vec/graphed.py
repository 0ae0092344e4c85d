"""A training step replayed as a HIP graph (small batches: the step is launch-bound).

At the reference's own batch shape (64 walks per step, configs/sge_sg_*.yaml) one step is a few
dozen microseconds of kernels — walker, SGNS pass 1, records sort, gather with the output
table's Adam fused, the input table's Adam on a side stream — and launching them one by one from
Python costs more than running them. ``GraphedStep`` captures the one-GPU step once per parity
of the input table's double buffer (two hipGraphs) and replays it.

What changes from step to step is kept in device memory (include/dw_hip.h, dw_step_scalars):
the walk id of the step's first walk (the Philox walker), the centre counter of its negatives
(SGNS pass 1) and the Adam scalars (both tables' updates). While a block is bound during
capture, those kernels read it instead of their by-value arguments. A graph replays `unroll`
steps: its first node, ``dw_step_scalars_expand``, writes the blocks of those steps from the
running block (and moves it past them) using a precomputed history of Adam scalars (float64 on
the host, rounded to float32 exactly as the eager launches pass them), plus the start nodes of
all their walks from the epoch's start list; one walker launch then generates those walks, and
step k's kernels are captured with block k bound. The kernels and their results are those of
the eager step (tests/test_gpu_graphed.py).
"""
from typing import Optional

import numpy as np
import torch

from shallow_encoders import _native
from shallow_encoders.word2vec.sharding import (OwnerLazyTables, ShardedTables, adam_scalars,
                                                hist_header, hist_row,
                                                owner_lazy_step, owner_lazy_steps,
                                                replicated_step)

_STEP_DTYPE = np.dtype([('walk_id0', '<u8'), ('noise_offset', '<u8'), ('step', '<i8'),
                        ('adam', '<f4', (8,))])   # == dw_step_scalars (56 bytes)


def adam_history(n_steps: int, lr: float, betas, eps: float, weight_decay: float) -> np.ndarray:
    """float32 [n_steps + 1, 8]: row s = Adam step s's scalars (dw_adam_dense order); row 0 the
    box header (sharding.hist_header)."""
    h = np.zeros((n_steps + 1, 8), dtype=np.float32)
    for s in range(1, n_steps + 1):
        h[s] = hist_row(s, lr, betas, eps, weight_decay)
    h[0] = hist_header(h, n_steps)
    return h


class GraphedStep:
    """``replicated_step`` on one GPU (ShardedTables; the out table's Adam fused into the records
    gather, or after the atomic scatter with ``scatter='atomic'``; the in table's Adam
    overlapped on the side stream, or with ``overlap_in=False`` both tables' Adam in one launch),
    captured with the walker in front of it.

    ``walker``: a Philox walker (rng='philox'; the replay walker's host-drawn uniforms cannot be
    captured); ``epoch_starts``: device int32 — walk w of the epoch starts at
    epoch_starts[w mod len]; the step trains walks ``first_walk_id + k*B ..``.
    ``n_steps``: how many training STEPS the Adam-scalar history covers (a replay runs
    ``unroll`` steps); ``replay`` raises before it would run past them.

    The walker's device tensors and the SGNS workspace are built before the capture (one
    eager walker launch into a scratch buffer — walks are a pure function of the walk id, so
    nothing is trained), and the walker's own walk-id counter is left where it was."""

    def __init__(self, tables: ShardedTables, walker, epoch_starts: torch.Tensor, B: int,
                 context_radius: int, neg_samples: int, *, seed: int, grad_scale: float,
                 loss_acc: torch.Tensor, status: torch.Tensor, first_walk_id: int,
                 n_steps: int, noise_offset: Optional[int] = None, scatter: str = 'sorted',
                 unroll: int = 1):
        if tables.world != 1 or not tables.can_fuse_out_adam():
            raise ValueError('GraphedStep: one GPU, HIP Adam')
        if epoch_starts.dtype != torch.int32 or epoch_starts.device != tables.device:
            raise ValueError('GraphedStep: epoch_starts must be int32 on the tables\' device')
        if unroll < 1:
            raise ValueError('GraphedStep: unroll must be >= 1')
        if getattr(walker, '_rng', None) != 'philox':
            raise ValueError("GraphedStep: the walker must be a Philox walker (rng='philox'); "
                             "rng='python' draws its uniforms on the host")
        self.unroll = int(unroll)
        self.t, self.walker = tables, walker
        dev = tables.device
        L = walker.length
        R, K = int(context_radius), int(neg_samples)
        self.B, self.centres = int(B), int(B) * (L - 2 * R)
        self.status, self.loss_acc = status, loss_acc
        self.epoch_starts = epoch_starts
        # the walks of all `unroll` steps of a graph come from ONE walker launch at its head:
        # walks are a pure function of the global walk id, and a latency-bound walker takes as
        # long for unroll*B walks as for B (the steps then read slices of the buffer)
        self.walks = torch.empty((self.unroll * self.B, L), dtype=torch.int32, device=dev)
        self.starts = torch.empty(self.unroll * self.B, dtype=torch.int32, device=dev)
        s1 = tables.step_count + 1                      # the Adam step the first replay applies
        hist = adam_history(s1 + n_steps + 2, tables.lr, tables.betas, tables.eps,
                            tables.weight_decay)
        self.hist = torch.from_numpy(hist).to(dev)
        blk = np.zeros(1, dtype=_STEP_DTYPE)
        blk['walk_id0'] = first_walk_id
        blk['noise_offset'] = (first_walk_id * (L - 2 * R) if noise_offset is None
                               else noise_offset)
        blk['step'] = s1
        blk['adam'][0] = hist[s1]
        self.block = torch.from_numpy(np.frombuffer(blk.tobytes(), dtype=np.uint8).copy()).to(dev)
        # the graph's steps' own blocks, written at its head by one dw_step_scalars_expand
        # (instead of one advance launch per step); step k's launches bind self._step_blk(k)
        self.step_blocks = torch.zeros(self.unroll * _STEP_DTYPE.itemsize, dtype=torch.uint8,
                                       device=dev)
        self._args = dict(seed=seed, grad_scale=grad_scale, scatter=scatter,
                          fuse_out_adam=scatter == 'sorted')
        self.R, self.K = R, K
        self.graphs = {}
        # Steps the scalar history covers: a graph whose first step is s needs rows s .. s+unroll
        # (the block it leaves for the next graph included), k_step_expand flags the rest
        self._hist_rows = int(hist.shape[0])
        # One-time builds happen here, not inside the capture: the walker's device tensors
        # (CSR, edges, adjacency hash, alias tables) via one eager launch into a scratch buffer,
        # and the records workspace of this step shape
        next_wid = walker._next_walk_id
        n_warm = min(self.B, int(epoch_starts.numel()))
        walker.walk_batch(epoch_starts[:n_warm], walk_id0=int(first_walk_id),
                          out=torch.empty((n_warm, L), dtype=torch.int32, device=dev),
                          check=False, status=torch.zeros(1, dtype=torch.int32, device=dev))
        walker._next_walk_id = next_wid
        from shallow_encoders.word2vec.sgns import _use_records, workspace_for
        if scatter == 'sorted' and _use_records(scatter, 2 * R, K, tables.V):
            workspace_for(self.centres, 2 * R, K, tables.V, dev)
        torch.cuda.synchronize(dev)
        # `unroll` consecutive steps per graph (one launch per `unroll` steps: at tiny batches
        # the gap between replays is as long as the step). One graph per parity of the in-table
        # double buffer (overlap_in) when a graph flips it (odd unroll); without the double
        # buffer (both tables' Adam in one in-place launch: the tiny-batch form) one graph.
        self._flips = tables.overlap_in and self.unroll % 2 == 1
        n_graphs = 2 if self._flips else 1
        for _ in range(n_graphs):
            parity = tables._cur_in
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, capture_error_mode='relaxed'):
                    self._body()
            finally:
                _native.call('dw_step_scalars_bind', None)
            self.graphs[parity] = g
        # the captures ran no step (host bookkeeping only; an even unroll ends on its parity)
        tables.step_count -= n_graphs * self.unroll
        walker._next_walk_id = next_wid   # the captured walker launch moved it (walk_id0=0)
        torch.cuda.synchronize(dev)

    def _step_blk(self, k: int) -> int:
        return self.step_blocks.data_ptr() + k * _STEP_DTYPE.itemsize

    def _body(self) -> None:
        """One graph: its steps' scalar blocks and start nodes (one launch; self.block moves
        past the graph), the walks of all its steps (one walker launch), then the steps."""
        t, dev, B = self.t, self.t.device, self.B
        with torch.cuda.device(dev):
            _native.call('dw_step_scalars_expand', _native.ptr(self.block), self._step_blk(0),
                         self.unroll, _native.ptr(self.hist), self.hist.shape[0], B,
                         self.centres, _native.ptr(self.status), _native.ptr(self.epoch_starts),
                         self.epoch_starts.numel(), _native.ptr(self.starts), self.starts.numel(),
                         _native.stream(dev))
        _native.call('dw_step_scalars_bind', self._step_blk(0))
        self.walker.walk_batch(self.starts, walk_id0=0, out=self.walks, check=False,
                               status=self.status)
        for k in range(self.unroll):
            _native.call('dw_step_scalars_bind', self._step_blk(k))
            replicated_step(t, self.walks[k * B:(k + 1) * B], self.R, self.K, noise_offset=0,
                            loss_acc=self.loss_acc, status=self.status, **self._args)

    def replay(self) -> None:
        """``unroll`` training steps (enqueued on the current stream); the tables' host
        bookkeeping (Adam step count, current in-table buffer) follows as the eager steps'
        would."""
        t = self.t
        if t.step_count + 1 + self.unroll >= self._hist_rows:
            raise RuntimeError(f'GraphedStep: the Adam-scalar history covers steps up to '
                               f'{self._hist_rows - 2}; build a new GraphedStep (n_steps) to go on')
        self.graphs[t._cur_in].replay()
        t.step_count += self.unroll
        if self._flips:
            t._next_in = 2 - t._cur_in
            t._cur_in = t._next_in

    def scalars(self) -> dict:
        """The device block (synchronises): walk_id0, noise_offset, step."""
        b = np.frombuffer(self.block.cpu().numpy().tobytes(), dtype=_STEP_DTYPE)[0]
        return {'walk_id0': int(b['walk_id0']), 'noise_offset': int(b['noise_offset']),
                'step': int(b['step'])}


# GraphedOwnerStep replays its side-first capture from this Adam step on (the in rows' lags, and
# so their catch-up, grow with the run; C3 / 64 walks: side-after 0.259 / 0.484 ms per step at
# steps 24-424 / 16,024-20,024, side-first 0.275 / 0.430)
SIDE_FIRST_FROM = 2000


class GraphedOwnerStep:
    """``owner_lazy_step`` on one GPU (OwnerLazyTables: the lazy exact Adam of the in table, and
    of the out table with ``lazy_out``) replayed as a HIP graph, with the walker in front of it:
    the reference's own batch shape on a large graph (C3 at 64 walks per step), where a step is
    ~40 kernel launches of a few microseconds each.

    As GraphedStep, what changes from step to step lives in the bound dw_step_scalars blocks
    (walk ids, the negatives' centre counter, the Adam scalars); the lazy kernels' step numbers
    (catch-ups, the out rows' claims, the lazy gather, the touched rows' update) are bound
    relative to each block (dw_step_scalars_bind_at), so the replays advance them on the device.
    The tables' Adam-scalar history is written ahead for ``n_steps`` steps before the capture,
    so begin_step copies nothing inside it.

    With the rows-major out step on one rank (OwnerLazyTables.pipeline_ok) the captured steps are
    pipelined (sharding.owner_lazy_steps): step k + 1's out-record placement, touch claim and
    catch-up run on side streams beside step k, and the graph's first step prepares its own.

    The tables must have run one eager step at this batch shape first (it allocates the
    touched-row, gather and workspace buffers the capture then reuses); the walker's device
    tensors are built here by one eager launch into a scratch buffer, and its walk-id counter
    is left where it was."""

    def __init__(self, tables: OwnerLazyTables, walker, epoch_starts: torch.Tensor, B: int,
                 context_radius: int, neg_samples: int, *, seed: int, grad_scale: float,
                 loss_acc: torch.Tensor, status: torch.Tensor, first_walk_id: int,
                 n_steps: int, unroll: int = 1):
        if not isinstance(tables, OwnerLazyTables) or tables.multi or tables.world != 1 \
                or not tables._hip():
            raise ValueError('GraphedOwnerStep: one GPU, OwnerLazyTables with the HIP Adam')
        if tables._touched is None or tables._G is None or tables.step_count < 1:
            raise ValueError('GraphedOwnerStep: run one eager owner_lazy_step at this batch shape '
                             'first (it allocates the buffers the capture reuses)')
        if epoch_starts.dtype != torch.int32 or epoch_starts.device != tables.device:
            raise ValueError('GraphedOwnerStep: epoch_starts must be int32 on the tables\' device')
        if unroll < 1:
            raise ValueError('GraphedOwnerStep: unroll must be >= 1')
        if getattr(walker, '_rng', None) != 'philox':
            raise ValueError("GraphedOwnerStep: the walker must be a Philox walker (rng='philox')")
        self.unroll = int(unroll)
        self.t, self.walker = tables, walker
        dev = tables.device
        L = walker.length
        R, K = int(context_radius), int(neg_samples)
        self.R, self.K = R, K
        self.B, self.centres = int(B), int(B) * (L - 2 * R)
        self.status, self.loss_acc, self.epoch_starts = status, loss_acc, epoch_starts
        self.seed, self.grad_scale = int(seed), float(grad_scale)
        self.walks = torch.empty((self.unroll * self.B, L), dtype=torch.int32, device=dev)
        self.starts = torch.empty(self.unroll * self.B, dtype=torch.int32, device=dev)
        s1 = tables.step_count + 1
        self._last = s1 + int(n_steps) + self.unroll   # history rows the replays may read
        tables.reserve_history(self._last)
        self._key = tables._hist_key
        hist = tables._hist
        self._hist_ptr = hist.data_ptr()   # captured by the graph's kernels
        blk = np.zeros(1, dtype=_STEP_DTYPE)
        blk['walk_id0'] = first_walk_id
        blk['noise_offset'] = first_walk_id * (L - 2 * R)
        blk['step'] = s1
        blk['adam'][0] = hist[s1].cpu().numpy()
        self.block = torch.from_numpy(np.frombuffer(blk.tobytes(), dtype=np.uint8).copy()).to(dev)
        self.step_blocks = torch.zeros(self.unroll * _STEP_DTYPE.itemsize, dtype=torch.uint8,
                                       device=dev)
        next_wid = walker._next_walk_id
        n_warm = min(self.B, int(epoch_starts.numel()))
        walker.walk_batch(epoch_starts[:n_warm], walk_id0=int(first_walk_id),
                          out=torch.empty((n_warm, L), dtype=torch.int32, device=dev),
                          check=False, status=torch.zeros(1, dtype=torch.int32, device=dev))
        walker._next_walk_id = next_wid
        torch.cuda.synchronize(dev)
        if tables.pipeline_ok(R, K):   # owner_lazy_steps' second buffers, outside the capture
            tables._pipe_alloc(self.B, L, R, K)
        steps0, lr0 = tables.step_count, len(tables._lr_hist)
        # Two captures of the same steps: the next step's preparation enqueued after this step's
        # out rows (early in a run) or before them (once the in rows' lags have grown, from
        # SIDE_FIRST_FROM steps on: the in-row catch-up is then the critical path and is
        # dispatched first; owner_lazy_steps side_first). (Captured and replayed on a
        # high-priority stream: 0.369 against 0.273 ms per step at C3 / 64 walks;
        # profiles/r06_pipe_order_ab.txt.)
        self.graph = torch.cuda.CUDAGraph()
        self.graph_late = None
        for late in ((False, True) if tables.pipeline_ok(R, K) else (False,)):
            g = torch.cuda.CUDAGraph() if late else self.graph
            try:
                with torch.cuda.graph(g, capture_error_mode='relaxed'):
                    self._body(side_first=late)
            finally:
                _native.call('dw_step_scalars_bind', None)
                tables.step_count = steps0          # the capture ran no step
                del tables._lr_hist[lr0:]
                walker._next_walk_id = next_wid
            if late:
                self.graph_late = g
        torch.cuda.synchronize(dev)

    def _step_blk(self, k: int) -> int:
        return self.step_blocks.data_ptr() + k * _STEP_DTYPE.itemsize

    def _body(self, side_first: bool = False) -> None:
        t, dev, B = self.t, self.t.device, self.B
        with torch.cuda.device(dev):
            _native.call('dw_step_scalars_expand', _native.ptr(self.block), self._step_blk(0),
                         self.unroll, _native.ptr(t._hist), self._last + 1, B, self.centres,
                         _native.ptr(self.status), _native.ptr(self.epoch_starts),
                         self.epoch_starts.numel(), _native.ptr(self.starts), self.starts.numel(),
                         _native.stream(dev))
        _native.call('dw_step_scalars_bind', self._step_blk(0))
        self.walker.walk_batch(self.starts, walk_id0=0, out=self.walks, check=False,
                               status=self.status)
        # the step numbers the lazy kernels get are relative to block k's (begin_step, inside
        # the steps, makes the host's count steps0 + k + 1 at step k)
        steps0 = t.step_count

        def bind(k):
            _native.call('dw_step_scalars_bind_at', self._step_blk(k), steps0 + k + 1)
        owner_lazy_steps(t, [self.walks[k * B:(k + 1) * B] for k in range(self.unroll)], self.R,
                         self.K, seed=self.seed, noise_offsets=[0] * self.unroll,
                         grad_scale=self.grad_scale, loss_acc=self.loss_acc, status=self.status,
                         bind=bind, side_first=side_first)

    def replay(self) -> None:
        """``unroll`` training steps (enqueued on the current stream); the tables' host
        bookkeeping (Adam step count) follows as the eager steps' would."""
        t = self.t
        if (t.lr, tuple(t.betas), t.eps, t.weight_decay) != self._key:
            raise RuntimeError('GraphedOwnerStep: the Adam hyper-parameters changed since the '
                               'capture; build a new GraphedOwnerStep')
        if t._hist.data_ptr() != self._hist_ptr:
            raise RuntimeError('GraphedOwnerStep: the tables\' Adam-scalar history was '
                               'reallocated since the capture; build a new GraphedOwnerStep')
        if t.step_count + self.unroll > self._last - self.unroll:
            raise RuntimeError(f'GraphedOwnerStep: the Adam-scalar history covers steps up to '
                               f'{self._last - self.unroll}; build a new GraphedOwnerStep '
                               f'(n_steps) to go on')
        late = self.graph_late is not None and t.step_count >= SIDE_FIRST_FROM
        (self.graph_late if late else self.graph).replay()
        t.step_count += self.unroll
        t._lr_hist.extend([t.lr] * self.unroll)

    def scalars(self) -> dict:
        """The device block (synchronises): walk_id0, noise_offset, step."""
        b = np.frombuffer(self.block.cpu().numpy().tobytes(), dtype=_STEP_DTYPE)[0]
        return {'walk_id0': int(b['walk_id0']), 'noise_offset': int(b['noise_offset']),
                'step': int(b['step'])}


class GraphedTrainerStep:
    """The user-facing training step (tools/train.py -> word2vec/fit.py: ``training_step`` on a
    device walk batch, then ``optimizer.step()``, trainer.py:131-152) replayed as a HIP graph of
    ``unroll`` steps, with the walker launch for all of them at its head: the reference configs'
    64-walk batches are launch-bound when stepped from Python one kernel at a time.

    Eligible (``eligible``): a RandomWalkDataset, ``manual_grads``, the HIP Adam holding exactly
    the two tables, no ``max_norm``. The walks are the Philox walker's, or (``rng='python'``) the
    reference's own: the walker's CPython random.random() stream generated in HBM by a generator
    whose state stays there across replays (graph/rng.py DeviceMT, the index read on the device),
    then the bit-exact replay walker. The negatives are the device Philox stream
    (``noise='device'``) or the reference's own (``noise='torch'``): torch.randint on the CPU
    generator's stream, likewise generated in HBM (DeviceMT.randint) for all the graph's steps at
    its head. The Python and torch generators get their states back on ``release_rng`` (fit calls
    it after the replays), exactly where the eager steps would have left them. The step is
    the trainer's own: the fused records step (the out table's Adam in the gather, the in
    table's on the side stream) or, for batches of <= 65,536 records, the atomic output-table
    scatter followed by ``optimizer.step()`` (bench.py's ``--scatter auto`` rule). What changes
    per step lives in the bound dw_step_scalars blocks (walk ids from the epoch's start list,
    the negatives' centre counter, the Adam scalars of the optimizer's history); the host
    bookkeeping (the optimizer's step counts, the trainer's centre counter, the dataset's
    position) follows each replay. ``unroll`` must be even: the fused step swaps the in table's
    buffers every step, so an even graph ends where it began.

    The tables, optimizer state and workspaces must exist (one eager step first: fit runs the
    epoch's first batch eagerly). ``replay`` returns the replayed steps' mean loss terms (device
    tensors), which fit pushes to the trainer's meter once per step they stand for."""

    @staticmethod
    def eligible(trainer, dataset) -> bool:
        from shallow_encoders.word2vec.optim import Adam
        walker = dataset.walk_generator
        opt = trainer.optimizer
        w_in, w_out = trainer.model.input_weight, trainer.model.output_weight
        if not (isinstance(opt, Adam) and opt.fuse_into_sgns and opt.zero_grad_in_step
                and len(opt.param_groups) == 1):
            return False
        mine = {id(p) for p in opt.param_groups[0]['params']}
        return (getattr(walker, '_rng', None) in ('philox', 'python')
                and trainer._noise_mode in ('device', 'torch')
                and trainer.manual_grads and trainer.model.max_norm is None
                and mine == {id(w_in), id(w_out)} and w_in.device.type == 'cuda'
                and trainer._context_radius is not None)

    def __init__(self, trainer, dataset, B: int, n_steps: int, unroll: int = 16,
                 scatter: str = 'auto'):
        """``scatter``: 'auto' (the atomic output-table scatter for <= 65,536 records, else the
        fused records step), 'records' (always the fused records step: the eager loop's kernels,
        so a graph trains what the eager steps train up to float-atomic order at chunk
        boundaries) or 'atomic'."""
        if scatter not in ('auto', 'records', 'atomic'):
            raise ValueError(f'GraphedTrainerStep: unknown scatter {scatter!r}')
        if unroll < 2 or unroll % 2:
            raise ValueError('GraphedTrainerStep: unroll must be even and >= 2')
        if not self.eligible(trainer, dataset):
            raise ValueError('GraphedTrainerStep: needs a walk-batch dataset, manual_grads and '
                             'the fusable HIP Adam (see eligible)')
        if not trainer.optimizer.can_fuse([trainer.model.input_weight,
                                           trainer.model.output_weight]):
            raise ValueError('GraphedTrainerStep: run one eager step first (gradient buffers, '
                             'Adam state)')
        from shallow_encoders.word2vec.sgns import _use_records
        self.trainer, self.dataset, self.walker = trainer, dataset, dataset.walk_generator
        self.unroll, self.B = int(unroll), int(B)
        w_in, w_out = trainer.model.input_weight, trainer.model.output_weight
        dev = w_in.device
        L = dataset.walk_length
        R, K = int(trainer._context_radius), int(trainer._neg_samples)
        self.R, self.K = R, K
        self.centres = self.B * (L - 2 * R)
        records = self.centres * 2 * R * (1 + K)
        from shallow_encoders.word2vec import exact
        if exact.enabled() and scatter == 'atomic':
            raise ValueError('GraphedTrainerStep: the deterministic mode needs the records step')
        # (the deterministic mode takes the records step: the atomic scatter sums in floats)
        self.scatter = ('atomic' if scatter == 'atomic' or (scatter == 'auto' and records <= 65_536
                                                            and not exact.enabled())
                        else None)   # (None: the fused step)
        if self.scatter is None and not _use_records('sorted', 2 * R, K, w_in.shape[0]):
            raise ValueError('GraphedTrainerStep: shape outside the records path')
        opt = trainer.optimizer
        group = opt.param_groups[0]
        self._params = (w_in, w_out)
        steps = {int(opt.state[p]['step'].item()) for p in self._params}
        if len(steps) != 1:
            raise ValueError('GraphedTrainerStep: the two tables are at different Adam steps')
        s1 = steps.pop() + 1
        self._key = (group['lr'], tuple(group['betas']), group['eps'], group['weight_decay'])
        self._last = s1 + int(n_steps)
        hist = adam_history(self._last + self.unroll + 1, group['lr'], group['betas'],
                            group['eps'], group['weight_decay'])
        self.hist = torch.from_numpy(hist).to(dev)
        self.epoch_starts = dataset._device_starts()
        first = dataset._index
        blk = np.zeros(1, dtype=_STEP_DTYPE)
        blk['walk_id0'] = dataset._epoch * len(dataset) + first
        blk['noise_offset'] = trainer._noise_offset
        blk['step'] = s1
        blk['adam'][0] = hist[s1]
        self.block = torch.from_numpy(np.frombuffer(blk.tobytes(), dtype=np.uint8).copy()).to(dev)
        self.step_blocks = torch.zeros(self.unroll * _STEP_DTYPE.itemsize, dtype=torch.uint8,
                                       device=dev)
        self.walks = torch.empty((self.unroll * self.B, L), dtype=torch.int32, device=dev)
        self.starts = torch.empty(self.unroll * self.B, dtype=torch.int32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.acc = torch.zeros(4, dtype=torch.float64, device=dev)
        # the reference's own streams, generated in HBM from generators held there across replays
        from shallow_encoders.graph.rng import DeviceMT
        self.mt_walks = self.mt_noise = self.uniforms = self.noise = None
        if self.walker._rng == 'python':
            self.uniforms = torch.empty(self.unroll * self.B * (L - 1), dtype=torch.float64,
                                        device=dev)
            self.mt_walks = DeviceMT.from_random(dev, device_index=True)
            self.mt_walks.reserve(self.uniforms.numel())
        if trainer._noise_mode == 'torch':
            self.V = int(w_in.shape[0])
            self.noise = torch.empty((self.unroll, self.centres, 2 * R, K), dtype=torch.int64,
                                     device=dev)
            self.mt_noise = DeviceMT.from_torch(dev, device_index=True)
            self.mt_noise.reserve(self.noise.numel(), self.V)
        torch.cuda.synchronize(dev)
        snap = ([opt.state[p]['step'].clone() for p in self._params], trainer._noise_offset,
                w_in.data_ptr())
        trainer._capture_acc, trainer._capture_scatter = self.acc, self.scatter
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph, capture_error_mode='relaxed'):
                self._body()
        finally:
            _native.call('dw_step_scalars_bind', None)
            trainer._capture_acc = trainer._capture_scatter = None
            for p, st in zip(self._params, snap[0]):   # the capture ran no step
                opt.state[p]['step'] = st
            trainer._noise_offset = snap[1]
        if w_in.data_ptr() != snap[2]:
            raise RuntimeError('GraphedTrainerStep: the in table did not end in its buffer')
        # the deterministic mode's int64 accumulators the captured kernels add into: held here,
        # so a replay never reaches freed memory whatever batch shapes the eager steps meet
        reg = getattr(trainer, '_exact', None)
        self._exact_refs = reg.live() if reg is not None else []
        torch.cuda.synchronize(dev)

    def _step_blk(self, k: int) -> int:
        return self.step_blocks.data_ptr() + k * _STEP_DTYPE.itemsize

    def _body(self) -> None:
        dev, B = self.acc.device, self.B
        self.acc.zero_()
        with torch.cuda.device(dev):
            _native.call('dw_step_scalars_expand', _native.ptr(self.block), self._step_blk(0),
                         self.unroll, _native.ptr(self.hist), self.hist.shape[0], B,
                         self.centres, _native.ptr(self.status), _native.ptr(self.epoch_starts),
                         self.epoch_starts.numel(), _native.ptr(self.starts), self.starts.numel(),
                         _native.stream(dev))
        _native.call('dw_step_scalars_bind', self._step_blk(0))
        if self.mt_walks is not None:   # the next unroll * B walks' uniforms, in walk order
            self.mt_walks.uniforms(self.uniforms.numel(), out=self.uniforms)
            self.walker.walk_batch(self.starts, uniforms=self.uniforms, out=self.walks,
                                   check=False, status=self.status)
        else:
            self.walker.walk_batch(self.starts, walk_id0=0, out=self.walks, check=False,
                                   status=self.status)
        if self.mt_noise is not None:   # every step's generate_noise_batch, in step order
            self.mt_noise.randint(self.V, self.noise.numel(), out=self.noise.view(-1))
        opt = self.trainer.optimizer
        try:
            for k in range(self.unroll):
                _native.call('dw_step_scalars_bind', self._step_blk(k))
                if self.noise is not None:
                    self.trainer._noise_override = self.noise[k]
                self.trainer.training_step(self.walks[k * B:(k + 1) * B])
                opt.step()
                opt.zero_grad()
        finally:
            self.trainer._noise_override = None

    def replay(self) -> dict:
        """``unroll`` training steps; returns their mean loss terms (device tensors)."""
        from shallow_encoders.word2vec.sgns import loss_terms
        t, opt = self.trainer, self.trainer.optimizer
        group = opt.param_groups[0]
        if (group['lr'], tuple(group['betas']), group['eps'], group['weight_decay']) != self._key:
            raise RuntimeError('GraphedTrainerStep: the optimizer hyper-parameters changed since '
                               'the capture; build a new one')
        step = int(opt.state[self._params[0]]['step'].item())
        if step + self.unroll > self._last:
            raise RuntimeError('GraphedTrainerStep: the Adam-scalar history is used up; build a '
                               'new one (n_steps)')
        self.graph.replay()
        for p in self._params:
            opt.state[p]['step'] += self.unroll
        t._noise_offset += self.unroll * self.centres
        self.dataset._index += self.unroll * self.B
        return loss_terms(self.acc, self.unroll * self.centres * 2 * self.R, self.K)

    def release_rng(self) -> None:
        """Hand the walk and noise streams back to CPython's ``random`` and torch's CPU
        generator (synchronises): after it they stand where the replayed steps, run eagerly, would
        have left them. Call it before anything else draws from either."""
        if self.mt_walks is not None:
            self.mt_walks.to_random()
        if self.mt_noise is not None:
            self.mt_noise.to_torch()


def epoch_starts_node_order(n_nodes: int, walks_per_node: int, device) -> torch.Tensor:
    """bench.py's start order: walk w starts at node w // walks_per_node + 1 (vocabulary id)."""
    ids = torch.arange(1, n_nodes + 1, dtype=torch.int32, device=device)
    return ids.repeat_interleave(walks_per_node)

