"""Inter-layer model parallelism (pipeline) over point-to-point RCCL / gloo.

Reference capability: MobileNetV2 split across 4 GPU
processes, activations forwarded and gradients returned through autograd
functions that wrap blocking ``dist.send/recv`` (``distributed_layers.py:7-62``,
loops in ``utils.py:34-210``, partition at ``model_parallel.py:101-104,
129-130,143-145``).  What changes here, MI355X-first:

* **Any world size.**  :func:`balanced_partition` cuts a model's atom
  sequence (``model.as_sequential()``) into contiguous stages minimising the
  largest stage cost (FLOPs measured with hooks, or parameters), instead of
  the reference's hard-coded 4-way slicing (defect 2); the stem keeps its ReLU
  (defect 3).
* **No host round-trips.**  The reference sends ``ndim`` and ``shape`` as fp32
  tensors before every payload and receives them with two device->host syncs
  (``distributed_layers.py:40-47``).  Here shapes are a static contract
  computed once per micro-batch size by a probe (:meth:`Pipeline._probe`), so
  every hop moves only the payload, in the activation dtype (bf16 works;
  reference defect 8 forced fp32 via ``torch.rand`` buffers).
* **Micro-batching.**  ``schedule="naive"`` reproduces the reference (one
  micro-batch, fully serialised); ``"gpipe"`` runs all forwards then all
  backwards over M micro-batches; ``"1f1b"`` (PipeDream-flush) interleaves
  one forward / one backward in steady state with batched send+recv pairs
  (one RCCL group each) so that stages overlap and activation memory is
  bounded by the stage depth.
* **Loss placement.**  ``loss_on="last"`` ships the targets to the last stage
  once per batch and returns [loss, top1, top5] to rank 0 (3 floats);
  ``loss_on="first"`` keeps the reference's ring (logits back to rank 0, loss
  there, dlogits to the last stage; gpipe/naive only).
* **Transport.**  :class:`~..comm.rccl.Communicator` -- RCCL send/recv on its
  own HIP stream on GPU (ordered with events, no blocking), gloo on CPU.
* **Device speed** (``graphs=True``, GPU, 1F1B, loss on the last stage).  Eagerly
  every micro-batch is hundreds of Python-dispatched kernel launches, so a
  64-image MobileNetV2 micro-batch costs as much host time as a whole
  512-image DDP step.  :class:`_StageGraphs` captures the
  stage's forward (with the loss and top-k statistics on the last stage) and
  backward once per in-flight slot as hipGraphs over static input / output /
  gradient buffers; a micro-batch is then a receive into the slot's static
  input, one forward replay, a send, a receive of the output gradient, one
  backward replay (parameter gradients accumulate in place inside the graph)
  and a send.  1F1B keeps at most ``S - r`` micro-batches in flight on stage
  r, so that many slots (memory pools) suffice.
* **Gradient accumulation in the kernels** (``kernel_grad_accum=True``): the
  weight-gradient kernels of the native ops add each micro-batch's parameter
  gradient straight into ``p.grad`` (:mod:`..ops.grad_accum`) instead of
  handing autograd a fresh tensor to add.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..comm.rccl import Communicator
from ..ops.grad_accum import accumulate_param_grads
from ..utils.graphs import no_gc_during_capture
from ..utils.profiling import trace_range


# --------------------------------------------------------------------------- #
# Partitioning
# --------------------------------------------------------------------------- #
def atom_costs(atoms: nn.Sequential, sample: torch.Tensor, kind: str = "flops") -> List[float]:
    """Per-atom cost: forward FLOPs of conv/linear layers (measured on `sample`) or params."""
    if kind == "params":
        return [float(sum(p.numel() for p in a.parameters())) or 1.0 for a in atoms]
    costs: List[float] = []
    flops = [0.0]

    def hook(mod, inp, out):
        if isinstance(mod, nn.Conv2d):
            k = mod.weight.numel() // mod.out_channels  # cin/groups * kh * kw
            flops[0] += 2.0 * out.numel() * k
        elif isinstance(mod, nn.Linear):
            flops[0] += 2.0 * out.numel() * mod.in_features
        else:
            flops[0] += float(out.numel()) if isinstance(out, torch.Tensor) else 0.0

    x = sample
    with torch.no_grad():
        was = [a.training for a in atoms]
        for a in atoms:
            a.eval()
        for a in atoms:
            hs = [m.register_forward_hook(hook) for m in a.modules()
                  if isinstance(m, (nn.Conv2d, nn.Linear)) or len(list(m.children())) == 0]
            flops[0] = 0.0
            x = a(x)
            for h in hs:
                h.remove()
            costs.append(max(flops[0], 1.0))
        for a, w in zip(atoms, was):
            a.train(w)
    return costs


def balanced_partition(costs: Sequence[float], stages: int) -> List[Tuple[int, int]]:
    """Contiguous split of `costs` into `stages` non-empty ranges minimising the max sum."""
    n = len(costs)
    if stages > n:
        raise ValueError(f"cannot cut {n} atoms into {stages} stages")
    pref = [0.0]
    for c in costs:
        pref.append(pref[-1] + c)
    INF = float("inf")
    # best[k][i] = minimal max-cost splitting first i atoms into k stages
    best = [[INF] * (n + 1) for _ in range(stages + 1)]
    arg = [[0] * (n + 1) for _ in range(stages + 1)]
    best[0][0] = 0.0
    for k in range(1, stages + 1):
        for i in range(k, n + 1):
            for j in range(k - 1, i):
                v = max(best[k - 1][j], pref[i] - pref[j])
                if v < best[k][i]:
                    best[k][i] = v
                    arg[k][i] = j
    bounds = []
    i = n
    for k in range(stages, 0, -1):
        j = arg[k][i]
        bounds.append((j, i))
        i = j
    return bounds[::-1]


def reference_partition(n_atoms: int, stages: int) -> List[Tuple[int, int]]:
    """The reference's MobileNetV2 cut (``model_parallel.py:101-104,129-130,143-145``)
    over our atoms (stem, 17 blocks, head, classifier): rank 0 = stem + blocks
    0..2, rank r in 1..ws-2 = blocks 6r-3..6r+2, last rank = the rest.  The
    reference only defines it for ws=4 (and leaves blocks unassigned otherwise,
    SURVEY §0 defect 2); here ws 2..4 are covered, the last rank taking every
    remaining block, and the stem keeps its ReLU (defect 3)."""
    if n_atoms != 20:
        raise ValueError("reference partition is defined for MobileNetV2's 20 atoms")
    if not 1 <= stages <= 4:
        raise ValueError("the reference cut covers 1..4 stages; use partition='balanced'")
    if stages == 1:
        return [(0, n_atoms)]
    bounds = [(0, 4)]
    for r in range(1, stages - 1):
        bounds.append((6 * r - 2, 6 * r + 4))
    bounds.append((bounds[-1][1], n_atoms))
    return bounds


# --------------------------------------------------------------------------- #
# P2P autograd functions (payload only; shapes are a static contract)
# --------------------------------------------------------------------------- #
class SendForwardRecvBackward(torch.autograd.Function):
    """forward: send x to `peer`, return x; backward: receive dL/dx from `peer`.

    Capability of the reference's ForwardSend_BackwardReceive
    (distributed_layers.py:7-26) without the 3-message shape handshake."""

    @staticmethod
    def forward(ctx, x, comm: Communicator, peer: int):
        ctx.comm, ctx.peer = comm, peer
        ctx.shape, ctx.dtype, ctx.device = x.shape, x.dtype, x.device
        with trace_range("pipe.send_fwd"):
            comm.send(x.contiguous(), peer)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        buf = torch.empty(ctx.shape, dtype=ctx.dtype, device=ctx.device)
        with trace_range("pipe.recv_bwd"):
            ctx.comm.recv(buf, ctx.peer)
            ctx.comm.wait()
        return buf, None, None


class RecvForwardSendBackward(torch.autograd.Function):
    """forward: receive the activation from `peer`; backward: send dL/dx to `peer`.

    Capability of the reference's generate_recv + ForwardReceive_BackwardSend
    (distributed_layers.py:40-62)."""

    @staticmethod
    def forward(ctx, anchor, shape, dtype, comm: Communicator, peer: int):
        ctx.comm, ctx.peer = comm, peer
        buf = torch.empty(shape, dtype=dtype, device=anchor.device)
        with trace_range("pipe.recv_fwd"):
            comm.recv(buf, peer)
            comm.wait()
        return buf

    @staticmethod
    def backward(ctx, g):
        with trace_range("pipe.send_bwd"):
            ctx.comm.send(g.contiguous(), ctx.peer)
        return None, None, None, None, None


def recv_activation(shape, dtype, device, comm: Communicator, peer: int) -> torch.Tensor:
    anchor = torch.empty(0, device=device, requires_grad=True)
    return RecvForwardSendBackward.apply(anchor, tuple(shape), dtype, comm, peer)


# --------------------------------------------------------------------------- #
# Pipeline engine
# --------------------------------------------------------------------------- #
class StepResult:
    """Per-step [loss, top1 %, top5 %] of one pipeline step.

    Holds the device tensor of the sums; the Python floats are materialised
    on first access (one host sync then), so a training loop that does not
    look at them every step never blocks on the pipeline (no
    per-step host round-trips).  ``loss_tensor`` is the 0-d device loss.
    """

    def __init__(self, loss: Optional[float] = None, top1: Optional[float] = None,
                 top5: Optional[float] = None, stats: Optional[torch.Tensor] = None,
                 batch: Optional[int] = None):
        self._vals = None if stats is not None else (loss, top1, top5)
        self._stats, self._batch = stats, batch

    def _get(self):
        if self._vals is None:
            s = self._stats.tolist()
            self._vals = (s[0], 100.0 * s[1] / self._batch, 100.0 * s[2] / self._batch)
        return self._vals

    @property
    def loss(self) -> Optional[float]:
        return self._get()[0]

    @property
    def top1(self) -> Optional[float]:
        return self._get()[1]

    @property
    def top5(self) -> Optional[float]:
        return self._get()[2]

    @property
    def loss_tensor(self) -> Optional[torch.Tensor]:
        return self._stats[0] if self._stats is not None else (
            None if self._vals[0] is None else torch.tensor(self._vals[0]))

    @property
    def valid(self) -> bool:
        return self._stats is not None or self._vals[0] is not None


def _topk_correct(logits: torch.Tensor, target: torch.Tensor, ks=(1, 5)) -> List[torch.Tensor]:
    maxk = min(max(ks), logits.shape[1])
    pred = logits.topk(maxk, 1, True, True).indices.t()
    correct = pred.eq(target.view(1, -1))
    return [correct[:min(k, maxk)].reshape(-1).float().sum() for k in ks]


class Pipeline:
    """One pipeline stage of a model cut across `comm.size` ranks.

    Every rank constructs the same full model (same seed) and keeps only its
    slice: ``Pipeline(model.as_sequential(), comm, sample_shape=(3, 32, 32))``.
    """

    def __init__(self, atoms: nn.Sequential, comm: Communicator, sample_shape: Sequence[int],
                 micro_batches: int = 1, schedule: str = "1f1b",
                 loss_fn: Optional[Callable] = None, loss_on: str = "last",
                 partition=None, balance: str = "flops",
                 device: Optional[torch.device] = None, dtype: torch.dtype = torch.float32,
                 channels_last: bool = False, static_batch: Optional[int] = None,
                 fail_fast: bool = True, graphs: bool = False, kernel_grad_accum: bool = True):
        if schedule not in ("naive", "gpipe", "1f1b"):
            raise ValueError(f"unknown schedule {schedule!r}")
        if loss_on not in ("last", "first"):
            raise ValueError("loss_on must be 'last' or 'first'")
        if loss_on == "first" and schedule == "1f1b":
            raise ValueError("loss_on='first' (reference ring) supports schedule naive/gpipe")
        self.comm = comm
        self.static_batch = static_batch  # batch-size contract shared by every rank (or None)
        self.rank, self.world = comm.rank, comm.size
        self.schedule = schedule
        self.micro_batches = 1 if schedule == "naive" else micro_batches
        if loss_fn is None:
            from ..ops.loss import cross_entropy as loss_fn  # fused HIP kernel on GPU
        self.loss_fn = loss_fn
        self.loss_on = loss_on if self.world > 1 else "last"
        self.device = torch.device(device) if device is not None else comm.device
        self.dtype = dtype
        self.channels_last = channels_last
        self.sample_shape = tuple(sample_shape)
        if partition == "reference":
            partition = reference_partition(len(atoms), self.world)
        elif partition is None or partition == "balanced":
            costs = atom_costs(atoms, torch.zeros((2,) + self.sample_shape), balance)
            partition = balanced_partition(costs, self.world)
        self.partition = partition
        self.is_first = self.rank == 0
        self.is_last = self.rank == self.world - 1
        self._tails = self._probe_tails(atoms)  # before our slice moves to the device
        lo, hi = partition[self.rank]
        self.module = nn.Sequential(*[atoms[i] for i in range(lo, hi)]).to(self.device)
        if dtype != torch.float32:
            from ..utils.precision import cast_model
            cast_model(self.module, dtype)
        if channels_last:
            self.module = self.module.to(memory_format=torch.channels_last)
        # an exception on one stage (e.g. rank 0 refusing a batch that breaks the
        # static contract) would leave the other stages blocked in a receive
        # forever: publish it so every rank exits non-zero (utils/debug.py)
        self.graphs = bool(graphs)
        # micro-batch gradient accumulation inside the weight-gradient kernels
        # (ops/grad_accum.py): no AccumulateGrad add per parameter per micro-batch
        self.kernel_grad_accum = bool(kernel_grad_accum)
        # one W^T per 1x1-conv weight per step, shared by the micro-batches'
        # data-gradient GEMMs (ops/wt_cache.py)
        from ..ops.conv1x1 import Conv1x1
        from ..ops.wt_cache import WTCache
        self._wt = WTCache(m.weight for m in self.module.modules() if isinstance(m, Conv1x1))
        self._graphs: Dict[int, "_StageGraphs"] = {}  # micro-batch size -> captured slots
        self.recaptures = 0  # forced re-captures of existing stage graphs (moved storage)
        self._failure = None
        if fail_fast and self.world > 1:
            from ..utils.debug import FailureBroadcast
            self._failure = FailureBroadcast(self.rank, self.world)

    def _guard(self):
        import contextlib
        return self._failure.guard() if self._failure is not None else contextlib.nullcontext()

    def close(self) -> None:
        """Stop the failure watcher (a finished pipeline)."""
        if self._failure is not None:
            self._failure.stop()

    # ---- static shape contract ------------------------------------------------
    def _probe_tails(self, atoms: nn.Sequential) -> List[Tuple[int, ...]]:
        """Per-stage output shape without the batch dim (computed locally on CPU from the
        full model every rank holds, so no shape message ever crosses the wire)."""
        tails = []
        x = torch.zeros((2,) + self.sample_shape)
        with torch.no_grad():
            for lo, hi in self.partition:
                for i in range(lo, hi):
                    a = atoms[i]
                    was = a.training
                    a.eval()
                    x = a(x)
                    a.train(was)
                tails.append(tuple(x.shape[1:]))
        return tails

    def _in_shape(self, mb: int) -> Tuple[int, ...]:
        return (mb,) + (self.sample_shape if self.is_first else self._tails[self.rank - 1])

    def _out_shape(self, mb: int) -> Tuple[int, ...]:
        return (mb,) + self._tails[self.rank]

    # ---- comm helpers ------------------------------------------------------------
    def _recv_fwd(self, mb: int) -> torch.Tensor:
        x = recv_activation(self._in_shape(mb), self.dtype, self.device, self.comm, self.rank - 1)
        return x

    def _split(self, t: torch.Tensor) -> List[torch.Tensor]:
        return list(torch.chunk(t, self.micro_batches, 0))

    def _mb_sizes(self, batch: int) -> List[int]:
        base = -(-batch // self.micro_batches)
        sizes, left = [], batch
        while left > 0:
            sizes.append(min(base, left))
            left -= sizes[-1]
        return sizes

    def _batch_size(self, inputs: Optional[torch.Tensor], batch_size: Optional[int] = None) -> int:
        """The step's batch.  Static contract (no message, no host sync): every
        rank passes ``batch_size`` (or the Pipeline was built with
        ``static_batch``); rank 0 checks its input against it.  Dynamic
        fallback: rank 0 forwards one int along the pipeline, which costs each
        later stage one host sync (the receive buffers are sized from it)."""
        if batch_size is None:
            batch_size = self.static_batch
        if batch_size is not None:
            if self.is_first and inputs is not None and inputs.shape[0] != batch_size:
                raise ValueError(f"pipeline batch contract is {batch_size} but rank 0 got "
                                 f"{inputs.shape[0]} (pass batch_size= for a ragged last batch)")
            return int(batch_size)
        t = torch.zeros(1, dtype=torch.int64, device=self.device)
        if self.is_first:
            t[0] = inputs.shape[0]
        if self.world > 1:
            if self.is_first:
                self.comm.send(t, 1)
            else:
                self.comm.recv(t, self.rank - 1)
                self.comm.synchronize()
                if not self.is_last:
                    self.comm.send(t, self.rank + 1)
        return int(t.item()) if not self.is_first else inputs.shape[0]

    # ---- compute helpers -----------------------------------------------------------
    def _prep_input(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.device, self.dtype, non_blocking=True)
        if self.channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        return x

    def _forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.module(x)

    # ---- public API -----------------------------------------------------------------
    def train_step(self, inputs: Optional[torch.Tensor] = None,
                   targets: Optional[torch.Tensor] = None, batch_size: Optional[int] = None) -> StepResult:
        """Forward + backward of one batch (inputs/targets needed on rank 0 only).
        Gradients accumulate in ``self.module``; step your stage optimizer after.
        ``batch_size`` (same on every rank) skips the batch-size message."""
        with self._guard():
            return self._train_step(inputs, targets, batch_size)

    def _train_step(self, inputs, targets, batch_size) -> StepResult:
        self.module.train()
        batch = self._batch_size(inputs, batch_size)
        sizes = self._mb_sizes(batch)
        if self.is_first:
            xs = list(torch.split(inputs, sizes, 0))
            ts = list(torch.split(targets, sizes, 0))
        else:
            xs, ts = None, None
        # targets to the last stage (loss_on="last")
        tgt = None
        if self.loss_on == "last":
            if self.world == 1:
                tgt = targets.to(self.device)
            elif self.is_first:
                self.comm.send(targets.to(self.device, torch.int64).contiguous(), self.world - 1)
            elif self.is_last:
                tgt = torch.empty(batch, dtype=torch.int64, device=self.device)
                self.comm.recv(tgt, 0)
                self.comm.wait()
            tgt_mbs = list(torch.split(tgt, sizes, 0)) if tgt is not None else None
        else:
            tgt_mbs = [t.to(self.device) for t in ts] if self.is_first else None
        stats = torch.zeros(3, dtype=torch.float64, device=self.device)
        import contextlib
        wt = contextlib.nullcontext()
        if self.device.type == "cuda" and len(self._wt) and self.micro_batches > 1:
            self._wt.refresh()  # the weights of this step, transposed once
            wt = self._wt.active()
        with accumulate_param_grads(self.kernel_grad_accum), wt:
            if self._graphed_ok(sizes):
                stats = self._run_1f1b_graphed(xs, tgt_mbs, sizes)
            elif self.schedule == "1f1b":
                self._run_1f1b(xs, tgt_mbs, sizes, stats)
            else:
                self._run_gpipe(xs, tgt_mbs, sizes, stats)
        return self._finish_stats(stats, batch)

    def _finish_stats(self, stats: torch.Tensor, batch: int) -> StepResult:
        holder = self.world - 1 if self.loss_on == "last" else 0
        if self.world > 1 and holder != 0:
            if self.is_last:
                self.comm.send(stats, 0)
            elif self.is_first:
                self.comm.recv(stats, holder)
                self.comm.wait()  # stream dependency only: the host does not block here
        if self.is_first or self.world == 1 or (self.rank == holder):
            return StepResult(stats=stats, batch=batch)
        return StepResult(None, None, None)

    def _fused_loss(self, y: torch.Tensor, t: torch.Tensor, stats: torch.Tensor) -> Optional[torch.Tensor]:
        """Loss / micro_batches with the statistics accumulated by the native
        cross-entropy kernels themselves (ops/loss.py cross_entropy_with_stats),
        when the stage uses the default loss on the GPU; else None."""
        from ..ops import loss as L
        if self.loss_fn is L.cross_entropy and stats.is_cuda and L._native_ce_ok(y, t):
            return L.cross_entropy_with_stats(y, t, 1.0 / self.micro_batches, stats)
        return None

    def _loss_and_stats(self, y: torch.Tensor, t: torch.Tensor, stats: torch.Tensor) -> torch.Tensor:
        fused = self._fused_loss(y, t, stats)
        if fused is not None:
            return fused
        logits = y.float()
        loss = self.loss_fn(logits, t) / self.micro_batches
        with torch.no_grad():
            c1, c5 = _topk_correct(logits, t)
            stats[0] += loss.detach().double()
            stats[1] += c1.double()
            stats[2] += c5.double()
        return loss

    # GPipe / naive: all forwards, then all backwards ----------------------------------
    def _run_gpipe(self, xs, tgts, sizes, stats):
        saved = []
        for m, mb in enumerate(sizes):
            x = self._prep_input(xs[m]) if self.is_first else self._recv_fwd(mb)
            y = self._forward(x)
            if self.is_last:
                if self.loss_on == "last":
                    saved.append(self._loss_and_stats(y, tgts[m], stats))
                else:  # ring: logits back to rank 0
                    saved.append(SendForwardRecvBackward.apply(y, self.comm, 0))
            else:
                saved.append(SendForwardRecvBackward.apply(y, self.comm, self.rank + 1))
            if self.is_first and self.loss_on == "first" and self.world > 1:
                saved[-1] = (saved[-1], m)
        if self.is_first and self.loss_on == "first" and self.world > 1:
            # receive logits of every micro-batch from the last stage, compute loss there
            losses = []
            for m, mb in enumerate(sizes):
                logits = recv_activation((mb,) + self._tails[-1], self.dtype, self.device,
                                         self.comm, self.world - 1)
                losses.append(self._loss_and_stats(logits, tgts[m], stats))
            for m in range(len(sizes)):
                losses[m].backward()  # sends dlogits to the last stage first (deadlock-free order)
                out, _ = saved[m]
                out.backward(torch.zeros_like(out))  # receives dL/dy from rank 1
            return
        for m in range(len(sizes)):
            out = saved[m]
            if self.is_last and self.loss_on == "last":
                out.backward()
            else:
                out.backward(torch.zeros_like(out))

    # 1F1B (PipeDream-flush) ------------------------------------------------------------
    def _run_1f1b(self, xs, tgts, sizes, stats):
        M = len(sizes)
        S, r = self.world, self.rank
        warm = min(S - r - 1, M)
        queue: List[Tuple[torch.Tensor, torch.Tensor]] = []
        fwd_i = 0

        def fwd_compute(x):
            nonlocal fwd_i
            m = fwd_i
            fwd_i += 1
            y = self._forward(x)
            if self.is_last:
                return x, self._loss_and_stats(y, tgts[m], stats)
            return x, y

        def get_input(m):
            if self.is_first:
                return self._prep_input(xs[m])
            buf = torch.empty(self._in_shape(sizes[m]), dtype=self.dtype, device=self.device)
            with trace_range("pipe.recv_fwd"):
                self.comm.recv(buf, r - 1)
                self.comm.wait()
            return buf.requires_grad_()

        def bwd(x, y, g):
            if self.is_last:
                y.backward()
            else:
                y.backward(g)
            return x.grad if not self.is_first else None

        for m in range(warm):
            x, y = fwd_compute(get_input(m))
            if not self.is_last:
                self.comm.send(y.detach().contiguous(), r + 1)
            queue.append((x, y))
        remaining = M - warm
        x_next = get_input(warm) if remaining > 0 else None
        b_i = 0
        for i in range(remaining):
            x, y = fwd_compute(x_next)
            queue.append((x, y))
            # send y forward, receive grad for the oldest in-flight micro-batch
            g = None
            if not self.is_last:
                g = torch.empty(self._out_shape(sizes[b_i]), dtype=self.dtype, device=self.device)
                with trace_range("pipe.send_fwd+recv_bwd"):
                    self.comm.batch_p2p([(y.detach().contiguous(), r + 1, True), (g, r + 1, False)])
                    self.comm.wait()
            xo, yo = queue.pop(0)
            gx = bwd(xo, yo, g)
            b_i += 1
            last_iter = i == remaining - 1
            if last_iter:
                if not self.is_first:
                    self.comm.send(gx.contiguous(), r - 1)
                x_next = None
            else:
                m_next = warm + i + 1
                if self.is_first:
                    x_next = get_input(m_next)
                else:
                    buf = torch.empty(self._in_shape(sizes[m_next]), dtype=self.dtype,
                                      device=self.device)
                    with trace_range("pipe.send_bwd+recv_fwd"):
                        self.comm.batch_p2p([(gx.contiguous(), r - 1, True), (buf, r - 1, False)])
                        self.comm.wait()
                    x_next = buf.requires_grad_()
        for _ in range(warm):
            xo, yo = queue.pop(0)
            g = None
            if not self.is_last:
                g = torch.empty(self._out_shape(sizes[b_i]), dtype=self.dtype, device=self.device)
                self.comm.recv(g, r + 1)
                self.comm.wait()
            gx = bwd(xo, yo, g)
            b_i += 1
            if not self.is_first:
                self.comm.send(gx.contiguous(), r - 1)

    # 1F1B on captured stage graphs ------------------------------------------------------
    def _graphed_ok(self, sizes) -> bool:
        # on CPU the same slot schedule runs on eager stand-ins of the graphs
        # (_EagerGraph): the gloo tests exercise it at any world size
        # on GPU only the bf16 native-kernel stage is captured: fp32 stages run
        # library convolutions (MIOpen), whose weight gradients do not survive
        # graph replay (profiles/README.md finding 48; a captured fp32 stage gave
        # garbage gradients from the second replay on, round 5)
        if self.device.type == "cuda" and (self.dtype != torch.bfloat16 or torch.cuda.is_current_stream_capturing()):
            return False
        return self.graphs and self.schedule == "1f1b" and self.loss_on == "last" and len(set(sizes)) == 1

    def _run_1f1b_graphed(self, xs, tgts, sizes) -> torch.Tensor:
        M = len(sizes)
        S, r = self.world, self.rank
        mb = sizes[0]
        depth = min(M, S - r)
        G = self._graphs.get(mb)
        if G is None or G.depth < depth or not G.valid():
            if G is not None and G.depth >= depth:
                # a re-capture forced by moved gradient / parameter / buffer
                # storage: legitimate after a re-homing, a silent slowdown when
                # it repeats (e.g. a torch optimizer's zero_grad(set_to_none=True)
                # every step): count it, say so once
                self.recaptures += 1
                if self.recaptures == 2:
                    import warnings
                    warnings.warn("Pipeline(graphs=True): stage graphs re-captured again because parameter "
                                  "gradients / parameters / buffers moved (set_to_none zero_grad?); every "
                                  "re-capture costs two eager iterations plus the slot captures",
                                  RuntimeWarning, stacklevel=2)
            G = self._graphs[mb] = _StageGraphs(self, mb, depth)
        G.stats.zero_()
        warm = min(S - r - 1, M)
        slot = lambda m: m % G.depth  # noqa: E731 - at most `depth` in flight (FIFO)

        def forward(m):
            k = slot(m)
            if self.is_first:
                G.inputs[k].copy_(xs[m])
            else:
                with trace_range("pipe.recv_fwd"):
                    self.comm.recv(G.inputs[k].detach(), r - 1)
                    self.comm.wait()
            if self.is_last:
                G.targets[k].copy_(tgts[m])
            G.fwd[k].replay()

        def backward(m, recv_grad: bool):
            k = slot(m)
            if not self.is_last and recv_grad:
                with trace_range("pipe.recv_bwd"):
                    self.comm.recv(G.gouts[k], r + 1)
                    self.comm.wait()
            G.bwd[k].replay()

        for m in range(warm):
            forward(m)
            if not self.is_last:
                self.comm.send(G.outs[slot(m)], r + 1)
        b = 0
        for m in range(warm, M):
            forward(m)
            if not self.is_last:
                # send this output, receive the oldest in-flight micro-batch's gradient
                with trace_range("pipe.send_fwd+recv_bwd"):
                    self.comm.batch_p2p([(G.outs[slot(m)], r + 1, True), (G.gouts[slot(b)], r + 1, False)])
                    self.comm.wait()
            backward(b, recv_grad=False)
            if not self.is_first:
                self.comm.send(G.inputs[slot(b)].grad, r - 1)
            b += 1
        while b < M:
            backward(b, recv_grad=True)
            if not self.is_first:
                self.comm.send(G.inputs[slot(b)].grad, r - 1)
            b += 1
        return G.stats.clone()  # the slots' statistics buffer is reused by the next step

    @torch.no_grad()
    def eval_step(self, inputs: Optional[torch.Tensor] = None,
                  targets: Optional[torch.Tensor] = None, batch_size: Optional[int] = None) -> StepResult:
        """Forward-only pass over the pipeline (reference val_* loops)."""
        with self._guard():
            return self._eval_step(inputs, targets, batch_size)

    def _eval_step(self, inputs, targets, batch_size) -> StepResult:
        self.module.eval()
        batch = self._batch_size(inputs, batch_size)
        sizes = self._mb_sizes(batch)
        stats = torch.zeros(3, dtype=torch.float64, device=self.device)
        tgt = None
        if self.world == 1:
            tgt = targets.to(self.device)
        elif self.is_first:
            self.comm.send(targets.to(self.device, torch.int64).contiguous(), self.world - 1)
        elif self.is_last:
            tgt = torch.empty(batch, dtype=torch.int64, device=self.device)
            self.comm.recv(tgt, 0)
            self.comm.wait()
        xs = list(torch.split(inputs, sizes, 0)) if self.is_first else None
        tg = list(torch.split(tgt, sizes, 0)) if tgt is not None else None
        for m, mb in enumerate(sizes):
            if self.is_first:
                x = self._prep_input(xs[m])
            else:
                x = torch.empty(self._in_shape(mb), dtype=self.dtype, device=self.device)
                self.comm.recv(x, self.rank - 1)
                self.comm.wait()
            y = self._forward(x)
            if self.is_last:
                logits = y.float()
                stats[0] += self.loss_fn(logits, tg[m]).double() * mb / batch
                c1, c5 = _topk_correct(logits, tg[m])
                stats[1] += c1.double()
                stats[2] += c5.double()
            else:
                self.comm.send(y.contiguous(), self.rank + 1)
        saved_mb = self.micro_batches
        self.micro_batches = 1  # stats[0] is already batch-weighted
        res = self._finish_stats_eval(stats, batch)
        self.micro_batches = saved_mb
        return res

    def _finish_stats_eval(self, stats, batch):
        if self.world > 1:
            if self.is_last:
                self.comm.send(stats, 0)
            elif self.is_first:
                self.comm.recv(stats, self.world - 1)
                self.comm.wait()
        if self.is_first:
            return StepResult(stats=stats, batch=batch)
        return StepResult(None, None, None)



class _EagerGraph:
    """CPU stand-in for a captured graph: ``replay()`` runs the function."""

    def __init__(self, fn):
        self.fn = fn

    def replay(self) -> None:
        self.fn()


class _StageGraphs:
    """``depth`` captured copies (slots) of one stage's forward and backward for
    micro-batch size ``mb`` (``Pipeline(graphs=True)``).

    Slot k owns a memory pool, a static input (the received activation, or the
    data on stage 0), a static output (sent on; NCHW-contiguous like the eager
    path's payload), a static output-gradient buffer and -- last stage -- the
    static targets and the micro-batch's loss / top-1 / top-5 accumulated into
    :attr:`stats` inside the forward graph.  The backward graph accumulates
    the parameter gradients IN PLACE into ``p.grad`` (which must exist and keep
    its storage: :meth:`valid` re-captures otherwise) and leaves the input
    gradient in ``inputs[k].grad``.  Capture follows ``make_graphed_callables``:
    two eager warm-up iterations on the capture stream (their effect on the
    running statistics and gradients is undone), then per slot the forward and
    the backward into one pool."""

    def __init__(self, pipe: "Pipeline", mb: int, depth: int):
        self.pipe, self.mb, self.depth = pipe, mb, depth
        dev = pipe.device
        self.params = [p for p in pipe.module.parameters() if p.requires_grad]
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)  # accumulated in place by the captured backward
        self.grad_ptrs = [p.grad.data_ptr() for p in self.params]
        self.param_ptrs = [p.data_ptr() for p in self.params]  # an optimizer may re-home them (flat buffers)
        # the captured forward updates the running statistics IN these buffers:
        # load_state_dict(assign=True) / module.to() would leave them behind
        self.buffer_keys = [(id(b), b.data_ptr()) for b in pipe.module.buffers()]
        self.stats = torch.zeros(3, dtype=torch.float64, device=dev)
        in_shape, out_shape = pipe._in_shape(mb), pipe._out_shape(mb)
        mk_in = lambda: torch.zeros(in_shape, dtype=pipe.dtype, device=dev)  # noqa: E731
        if pipe.is_first and pipe.channels_last and len(in_shape) == 4:
            mk_in = lambda: torch.zeros(in_shape, dtype=pipe.dtype, device=dev).contiguous(  # noqa: E731
                memory_format=torch.channels_last)
        self.inputs = [mk_in().requires_grad_(not pipe.is_first) for _ in range(depth)]
        self.targets = [torch.zeros(mb, dtype=torch.int64, device=dev) for _ in range(depth)]
        self.gouts = [torch.zeros(out_shape, dtype=pipe.dtype, device=dev) for _ in range(depth)]
        self.outs: List[Optional[torch.Tensor]] = []
        self.fwd: List[torch.cuda.CUDAGraph] = []
        self.bwd: List[torch.cuda.CUDAGraph] = []
        if dev.type == "cuda":
            self.stream = torch.cuda.Stream(device=dev)
            self._capture()
        else:
            self._eager_slots()

    def _eager_slots(self) -> None:
        """CPU: the replays re-run forward / backward eagerly with the same static
        buffers and in-place semantics (the input gradient is replaced, the
        parameter gradients accumulate, the last stage's stats accumulate)."""
        live = [None] * self.depth

        def fwd(k):
            out = self._forward(k)
            live[k] = out
            if self.outs[k] is not None:
                with torch.no_grad():
                    self.outs[k].copy_(out)

        def bwd(k):
            self.inputs[k].grad = None
            self._backward(k, live[k])
            live[k] = None

        shape = self.pipe._out_shape(self.mb)
        for k in range(self.depth):
            self.fwd.append(_EagerGraph(lambda k=k: fwd(k)))
            self.bwd.append(_EagerGraph(lambda k=k: bwd(k)))
            self.outs.append(None if self.pipe.is_last else
                             torch.zeros(shape, dtype=self.pipe.dtype, device=self.pipe.device))

    def _forward(self, k: int) -> torch.Tensor:
        pipe = self.pipe
        y = pipe.module(self.inputs[k])
        if not pipe.is_last:
            return y.contiguous()  # the wire layout of the eager path (its backward: a copy)
        fused = pipe._fused_loss(y, self.targets[k], self.stats)
        if fused is not None:
            return fused
        logits = y.float()
        loss = pipe.loss_fn(logits, self.targets[k]) / pipe.micro_batches
        with torch.no_grad():
            c1, c5 = _topk_correct(logits, self.targets[k])
            self.stats[0] += loss.detach().double()
            self.stats[1] += c1.double()
            self.stats[2] += c5.double()
        return loss

    def _backward(self, k: int, out: torch.Tensor) -> None:
        if self.pipe.is_last:
            out.backward()
        else:
            out.backward(self.gouts[k])

    def _capture(self) -> None:
        pipe = self.pipe
        bufs = [b for b in pipe.module.buffers()]
        saved_b = [b.detach().clone() for b in bufs]
        saved_g = [p.grad.detach().clone() for p in self.params]
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(pipe.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # lazy library initialisation outside the capture
                self._backward(0, self._forward(0))
        torch.cuda.current_stream(pipe.device).wait_stream(s)
        with torch.no_grad():
            for b, v in zip(bufs, saved_b):
                b.copy_(v)
            for p, v in zip(self.params, saved_g):
                p.grad.copy_(v)
            self.stats.zero_()
        for x in self.inputs:
            x.grad = None
        torch.cuda.synchronize(pipe.device)
        # no Python garbage collection inside the captures (utils/graphs.py)
        with no_gc_during_capture(pipe.device):
            for k in range(self.depth):
                pool = torch.cuda.graph_pool_handle()
                gf, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                with torch.cuda.graph(gf, pool=pool, stream=s):
                    out = self._forward(k)
                with torch.cuda.graph(gb, pool=pool, stream=s):
                    self._backward(k, out)
                self.fwd.append(gf)
                self.bwd.append(gb)
                self.outs.append(out.detach() if not pipe.is_last else None)
        torch.cuda.synchronize(pipe.device)

    def valid(self) -> bool:
        """The captured backward adds into the gradient storage seen at capture,
        and the captured forward reads / updates the same parameter and buffer
        tensors."""
        return (all(p.grad is not None and p.grad.data_ptr() == g and p.data_ptr() == d
                    for p, g, d in zip(self.params, self.grad_ptrs, self.param_ptrs))
                and [(id(b), b.data_ptr()) for b in self.pipe.module.buffers()] == self.buffer_keys)
