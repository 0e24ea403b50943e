"""DistributedDataParallel over the native C++ Reducer and RCCL.

Parity target: upstream ``DistributedDataParallel`` as studied in the
reference README (Readme.md:145-157) -- the reference
itself contains no DDP code.  Public API kept call-compatible for the common
subset: ``DistributedDataParallel(module, device_ids=None, output_device=None,
broadcast_buffers=True, bucket_cap_mb=25, find_unused_parameters=False,
gradient_as_bucket_view=True, ...)``, ``no_sync()``, ``register_comm_hook``,
``.module``.

MI355X-first design (one process per GPU, torchrun):
  * gradients are bucket views of one flat buffer per dtype; buckets (25 MB
    default, 1 MB first bucket -- SURVEY.md §5.8 sizing for 7 xGMI links) are
    all-reduced by C++ hooks with RCCL ``ncclAvg`` on a dedicated HIP
    stream while backward continues on the compute stream;
  * ``flat_parameters=True`` additionally makes every parameter a view into a
    flat parameter buffer laid out exactly like the gradient buckets, so
    :class:`~..ops.optim.FlatSGD` updates the whole model in one kernel;
  * module buffers (BN running stats) are held flat too and broadcast from
    rank 0 with ONE collective per forward (``broadcast_buffers``);
  * after the first backward the buckets are rebuilt in the observed
    autograd-ready order of rank 0 (all ranks adopt the same order).
"""
from __future__ import annotations

import contextlib
import os
import time
from typing import Any, Callable, Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.env import single_rank_comm
from .. import _native
from ..comm.rccl import Communicator, default_communicator, verify_comm_layout
from ..ops import flat as flatops
from ..utils.profiling import trace_range

_MB = 1024 * 1024


def _tensors_in(obj) -> List[torch.Tensor]:
    out: List[torch.Tensor] = []
    if isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            out.extend(_tensors_in(o))
    elif isinstance(obj, dict):
        for o in obj.values():
            out.extend(_tensors_in(o))
    return out


def _bucket_assignment_py(params: Sequence[torch.Tensor], order: Sequence[int], cap: int,
                          first_cap: int) -> List[List[int]]:
    """Pure-Python bucket assignment used when an explicit order is given."""
    out: List[List[int]] = []
    open_: Dict[Any, List] = {}
    first_done = False
    for i in order:
        p = params[i]
        key = (p.dtype, p.device)
        idxs, size = open_.get(key, ([], 0))
        idxs = idxs + [i]
        size += ((p.numel() + 7) // 8 * 8) * p.element_size()
        limit = cap if first_done else first_cap
        if size >= limit:
            out.append(idxs)
            open_[key] = ([], 0)
            first_done = True
        else:
            open_[key] = (idxs, size)
    for idxs, _ in open_.values():
        if idxs:
            out.append(idxs)
    return out


class _PyHookBackend:
    """Python comm hook adapter: average all-reduce over a process group.

    With ``timing`` on it keeps host timestamps per bucket (the gloo / CPU form
    of the RCCL backend's event timing): the launch (bucket ready), the start
    and end of its wait.  Waits run in bucket order once backward has finished,
    so the first wait marks the end of backward and the last one the end of the
    exposed communication tail."""

    def __init__(self, group, world: int, fp32_accum: bool = False):
        self.group = group
        self.world = world
        self.fp32_accum = fp32_accum
        self.timing = False
        self._t = {}
        self.last = None

    def __call__(self, index: int, bucket: torch.Tensor):
        red = bucket.float() if self.fp32_accum and bucket.dtype in (torch.bfloat16, torch.float16) else bucket
        work = dist.all_reduce(red, group=self.group, async_op=True)
        world = self.world
        backend = self
        if self.timing:
            self._t[index] = [time.perf_counter(), 0.0, 0.0]

        class _H:
            def wait(self_inner):
                t = backend._t.get(index) if backend.timing else None
                if t is not None:
                    t[1] = time.perf_counter()
                work.wait()
                if red is bucket:
                    bucket.div_(world)
                else:
                    bucket.copy_(red.div_(world))
                if t is not None:
                    t[2] = time.perf_counter()
                    if index == max(backend._t):
                        backend._close()

        return _H()

    def _close(self) -> None:
        ts = [self._t[i] for i in sorted(self._t)]
        self._t = {}
        if not ts:
            return
        ready_done = [1e3 * (t[2] - t[0]) for t in ts]
        coll = [ready_done[0]] + [min(ready_done[i], 1e3 * (ts[i][2] - ts[i - 1][2])) for i in range(1, len(ts))]
        self.last = ready_done + coll + [1e3 * (ts[-1][2] - ts[0][1])]


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, device_ids: Optional[Sequence[int]] = None,
                 output_device: Optional[int] = None, dim: int = 0,
                 broadcast_buffers: bool = True, process_group: Optional[dist.ProcessGroup] = None,
                 bucket_cap_mb: float = 25.0, find_unused_parameters: bool = False,
                 gradient_as_bucket_view: bool = True, static_graph: bool = False,
                 first_bucket_mb: float = 1.0, flat_parameters: bool = False,
                 rebuild_buckets: bool = True, communicator: Optional[Communicator] = None,
                 reduce_dtype: Optional[torch.dtype] = None):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("DistributedDataParallel requires torch.distributed to be initialised "
                               "(see distributed_model_parallel_amd.utils.env.init_distributed)")
        if not gradient_as_bucket_view:
            # Kept for signature compatibility: gradients are ALWAYS bucket views here,
            # which is strictly cheaper (no copy in or out of buckets).
            pass
        self.module = module
        self.dim = dim
        self.group = process_group
        self.world_size = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.broadcast_buffers = broadcast_buffers
        self.find_unused_parameters = find_unused_parameters
        self.static_graph = static_graph
        self.require_backward_grad_sync = True
        self.require_forward_param_sync = True
        # reduce_dtype=torch.float32: bf16 / fp16 buckets are averaged through an
        # fp32 copy (one rounding instead of one per ring hop; 2x the bytes)
        if reduce_dtype not in (None, torch.float32):
            raise ValueError("reduce_dtype must be None (the gradient dtype) or torch.float32")
        self.reduce_fp32 = reduce_dtype == torch.float32
        self.bucket_cap = int(bucket_cap_mb * _MB)
        self.first_bucket_cap = int(first_bucket_mb * _MB)
        self._rebuild_pending = rebuild_buckets and not static_graph
        self._iteration = 0
        self._layout_version = 0
        self._flat_params: Optional[List[torch.Tensor]] = None
        self.buffer_broadcasts = 0  # collectives issued for module buffers (diagnostics)

        params = []
        seen = set()
        for p in module.parameters():
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                params.append(p)
        if not params:
            raise RuntimeError("DistributedDataParallel: module has no parameters that require grad")
        self._params = params
        dev = params[0].device
        self.device = dev
        for p in params:
            if p.device != dev:
                raise ValueError("DistributedDataParallel expects a single-device module "
                                 "(one process per GPU)")
        self.device_ids = list(device_ids) if device_ids is not None else (
            [dev.index] if dev.type == "cuda" else None)
        self.output_device = output_device

        if dev.type == "cuda":
            self.comm = communicator or (default_communicator(dev) if process_group is None
                                          else Communicator(dev, process_group, purpose="ddp"))
        else:
            self.comm = communicator or Communicator(dev, process_group, purpose="ddp")
        verify_comm_layout("DistributedDataParallel", process_group)

        self._verify_params_across_ranks()
        self._sync_module_states()

        C = _native.native()
        if C is None:
            raise RuntimeError("DistributedDataParallel needs the native extension (_C); build it "
                               "with `python csrc/build.py`")
        self._C = C
        buckets = C.compute_bucket_assignment(params, self.bucket_cap, self.first_bucket_cap)
        # The reducer creates the parameters' AccumulateGrad nodes: create them on
        # the weight-gradient side stream, so the weight-gradient kernels, the
        # bucket flushes and the all-reduce launches all run off the data-gradient
        # chain (ops/wgrad_stream.py)
        from ..ops import wgrad_stream
        with wgrad_stream.creating_on_side(dev):
            self.reducer = C.Reducer(params, buckets, self._make_backend(), find_unused_parameters)
        self.async_wgrad_params = wgrad_stream.mark_bound(params) if dev.type == "cuda" else 0
        self._buffers_flat: Optional[List[torch.Tensor]] = None
        if flat_parameters:
            self._install_flat_params()
        self._setup_flat_buffers()

    # ------------------------------------------------------------------ #
    def _make_backend(self):
        C = _native.native()
        self._timing_src = None  # the object whose timing the bench reads
        if self.world_size == 1 and not single_rank_comm():
            # averaging over one rank is the identity: no collective to launch
            self.comm_backend = "none(world_size=1)"
            return C.NullReduceBackend()
        if self.comm.native is not None:
            self.comm_backend = "rccl"
            b = C.RcclReduceBackend(self.comm.native, fp32_accum=self.reduce_fp32)
            self._timing_src = b
            return b
        self.comm_backend = "process_group"
        hook = _PyHookBackend(self.group, self.world_size, self.reduce_fp32)
        self._timing_src = hook
        return C.PyReduceBackend(hook)

    # ------------------------------------------------------------------ #
    def enable_comm_timing(self, on: bool = True) -> None:
        """Time every bucket's all-reduce and the exposed communication tail of
        each backward (HIP events on the RCCL path, host clocks on a process
        group); read with ``comm_timing()``."""
        src = self._timing_src
        if src is None:
            return
        if isinstance(src, _PyHookBackend):
            src.timing = bool(on)
        else:
            src.set_timing(bool(on))

    def comm_timing(self) -> dict:
        """The last backward's communication accounting (the reference's
        "bucketed ring all-reduce overlapped with backward", Readme.md:145-157,
        made measurable): per bucket (launch order) the ms from the bucket being
        ready to its all-reduce done and the all-reduce's own ms, and the exposed
        tail -- ms from the end of backward until every bucket is reduced."""
        out = {"backend": self.comm_backend}
        src = self._timing_src
        if src is None:
            return out
        if isinstance(src, _PyHookBackend):
            vals, out["source"] = src.last, "host_clock"
        else:
            vals, out["source"] = list(src.last_timing()), "hip_events"
        if not vals:
            return out
        n = (len(vals) - 1) // 2
        r = lambda xs: [round(float(x), 3) for x in xs]  # noqa: E731
        out.update({"buckets_timed": n, "ready_to_done_ms": r(vals[:n]), "allreduce_ms": r(vals[n:2 * n]),
                    "allreduce_ms_total": round(float(sum(vals[n:2 * n])), 3),
                    "exposed_tail_ms": round(float(vals[-1]), 3)})
        return out

    def register_comm_hook(self, state: Any, hook: Callable) -> None:
        """hook(state, bucket_tensor) -> torch.futures.Future (result ignored; the
        hook must leave the reduced gradient in the bucket tensor)."""
        def adapter(index, bucket):
            # buckets are launched in index order (csrc/ddp/reducer.cpp
            # in-order launch): the last one reduced has the highest index
            fut = hook(state, _Bucket(index, bucket, len(self.reducer.buckets())))

            class _H:
                def wait(self_inner):
                    res = fut.wait()
                    if isinstance(res, (list, tuple)):
                        res = res[0]
                    if isinstance(res, torch.Tensor) and res.data_ptr() != bucket.data_ptr():
                        bucket.copy_(res)
            return _H()
        self.reducer.set_backend(self._C.PyReduceBackend(adapter))

    # ------------------------------------------------------------------ #
    def _verify_params_across_ranks(self) -> None:
        if self.world_size == 1:
            return
        import zlib
        sig = torch.tensor([len(self._params)] + [
            zlib.crc32(repr((tuple(p.shape), str(p.dtype), i)).encode()) % (2 ** 24)
            for i, p in enumerate(self._params)], dtype=torch.float64)
        s = torch.tensor([sig.sum().item(), float(len(self._params))], dtype=torch.float64,
                         device=self.device if self.device.type == "cuda" else "cpu")
        mx = s.clone()
        mn = -s.clone()
        self.comm.all_reduce(mx, "max")
        self.comm.all_reduce(mn, "max")
        self.comm.synchronize()
        if not torch.equal(mx, -mn):
            raise RuntimeError("DistributedDataParallel: parameter shapes/dtypes differ across ranks")

    @torch.no_grad()
    def _broadcast_coalesced(self, tensors: Sequence[torch.Tensor], root: int = 0) -> None:
        if self.world_size == 1 or not tensors:
            return
        for (_dt, _dev), idxs in flatops.group_by_dtype(tensors).items():
            ts = [tensors[i] for i in idxs]
            flat = flatops.flatten(ts)
            self.comm.broadcast(flat, root)
            self.comm.wait()
            flatops.unflatten_into(flat, ts)

    def _sync_module_states(self) -> None:
        states = [p.detach() for p in self.module.parameters()] + \
                 [b for b in self.module.buffers()]
        self._broadcast_coalesced(states, 0)

    def _install_flat_params(self) -> None:
        """Make parameters views of flat buffers laid out like the grad buckets."""
        flats_g = self.reducer.group_flats()
        layout = self.reducer.layout()
        new_flats = [torch.zeros_like(g) for g in flats_g]
        with torch.no_grad():
            for p, (g, off) in zip(self._params, layout):
                view = new_flats[g].as_strided(p.shape, p.stride(), off)
                view.copy_(p.detach())
                p.data = view
        self._flat_params = new_flats
        self._layout_version += 1

    def _setup_flat_buffers(self) -> None:
        """Hold float buffers (BN running stats) in one flat tensor per dtype so the
        per-forward broadcast is a single collective."""
        bufs = [b for b in self.module.buffers() if b.is_floating_point() or b.dtype == torch.long]
        if not bufs:
            self._buffers_flat = []
            return
        groups = flatops.group_by_dtype(bufs)
        self._buffers_flat = []
        for (_dt, _dev), idxs in groups.items():
            ts = [bufs[i] for i in idxs]
            flat = flatops.flatten(ts)
            offs, _ = flatops.flat_layout(ts)
            for t, o in zip(ts, offs):
                t.data = flat.narrow(0, o, t.numel()).view(t.shape)
            self._buffers_flat.append(flat)

    # ------------------------------------------------------------------ #
    @property
    def layout_version(self) -> int:
        return self._layout_version

    def flat_groups(self):
        """[(param_flat, grad_flat)] per dtype group (requires flat_parameters)."""
        if self._flat_params is None:
            raise RuntimeError("flat_groups() needs DistributedDataParallel(..., flat_parameters=True)")
        return list(zip(self._flat_params, self.reducer.group_flats()))

    def param_layout(self):
        return self.reducer.layout()

    def bucket_summary(self) -> dict:
        """Bucket layout facts for diagnostics / the multi-rank rehearsal: the
        parameter indices per bucket (launch order), their MB, a digest, and
        whether the ready-order rebuild has happened."""
        import zlib
        buckets = [[int(i) for i in b] for b in self.reducer.buckets()]
        mb = [round(sum(self._params[i].numel() * self._params[i].element_size() for i in b) / _MB, 3)
              for b in buckets]
        return {"buckets": len(buckets), "bucket_mb": mb, "digest": zlib.crc32(repr(buckets).encode()),
                "rebuilt": not self._rebuild_pending}

    def _maybe_rebuild_buckets(self) -> None:
        if not self._rebuild_pending or self._iteration < 1:
            return
        self._rebuild_pending = False
        order = list(self.reducer.ready_order())
        n = len(self._params)
        # rank 0's observed order; params never seen go last in reverse registration order
        t = torch.full((n,), -1, dtype=torch.float64,
                       device=self.device if self.device.type == "cuda" else "cpu")
        if order:
            t[: len(order)] = torch.tensor(order, dtype=torch.float64)
        self.comm.broadcast(t, 0)
        self.comm.synchronize()
        order = [int(v) for v in t.tolist() if v >= 0]
        rest = [i for i in reversed(range(n)) if i not in set(order)]
        order = order + rest
        new = _bucket_assignment_py(self._params, order, self.bucket_cap, self.first_bucket_cap)
        if new == [list(b) for b in self.reducer.buckets()]:
            return
        old_layout = self.reducer.layout()
        self.reducer.rebuild(new)
        if self._flat_params is not None:
            old_flats = self._flat_params
            self._install_flat_params()
            del old_flats
        self._layout_version += 1
        self._last_old_layout = old_layout

    def zero_grad(self) -> None:
        """Zero all gradients in place (one fill per dtype group)."""
        self.reducer.zero_grad()

    @contextlib.contextmanager
    def no_sync(self):
        old = self.require_backward_grad_sync
        self.require_backward_grad_sync = False
        try:
            yield
        finally:
            self.require_backward_grad_sync = old

    def forward(self, *inputs, **kwargs):
        if torch.is_grad_enabled() and self.require_backward_grad_sync:
            self._maybe_rebuild_buckets()
        if self.broadcast_buffers and self.world_size > 1 and self._buffers_flat:
            with trace_range("ddp.broadcast_buffers"):
                for f in self._buffers_flat:  # one collective per buffer dtype group
                    self.comm.broadcast(f, 0)
                    self.buffer_broadcasts += 1
                self.comm.wait()
        with trace_range("ddp.forward"):
            out = self.module(*inputs, **kwargs)
        if torch.is_grad_enabled() and self.require_backward_grad_sync:
            outs = _tensors_in(out) if self.find_unused_parameters else []
            self.reducer.prepare_for_backward(outs)
            self._iteration += 1
        else:
            self.reducer.disarm()
        return out

    # state_dict passes through to the wrapped module under "module." like upstream
    def train(self, mode: bool = True):
        super().train(mode)
        return self


class _Bucket:
    """Object handed to comm hooks (mirrors upstream GradBucket's essentials).

    ``index()`` is the launch position: bucket 0 (the parameters whose
    gradients are ready first in backward) is reduced first, and ``is_last()``
    is true for the bucket reduced last in the iteration -- upstream's meaning
    (a hook that flushes per-iteration state on the last bucket sees every
    other bucket first)."""

    def __init__(self, index: int, buffer: torch.Tensor, num_buckets: int):
        self._index = index
        self._buffer = buffer
        self._num = num_buckets

    def index(self) -> int:
        return self._index

    def buffer(self) -> torch.Tensor:
        return self._buffer

    def is_last(self) -> bool:
        return self._index == self._num - 1


def allreduce_hook(group):
    """Default comm hook (average all-reduce) for register_comm_hook."""
    def hook(state, bucket: _Bucket):
        ws = dist.get_world_size(group)
        t = bucket.buffer()
        fut = dist.all_reduce(t, group=group, async_op=True).get_future()
        return fut.then(lambda f: f.value()[0].div_(ws))
    return hook


def bf16_compress_hook(group):
    """Compress fp32 buckets to bf16 for the all-reduce (halves xGMI bytes)."""
    def hook(state, bucket: _Bucket):
        ws = dist.get_world_size(group)
        t = bucket.buffer()
        c = t.to(torch.bfloat16)
        fut = dist.all_reduce(c, group=group, async_op=True).get_future()

        def done(f):
            t.copy_(f.value()[0].float().div_(ws))
            return t
        return fut.then(done)
    return hook
