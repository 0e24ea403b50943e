"""DataParallel replicas as hipGraphs (``DataParallel(..., graphs=True)``).

The reference's DataParallel runs one Python thread per replica and warns it
"may cause threshing" (Readme.md:10): every replica's forward and backward is
thousands of Python-dispatched kernel launches, and the threads serialise on
the GIL (measured round 3: ResNet-50, 4 replicas of 64 images, 69.7 ms per
step vs 23.2 ms for DDP on the same 256 images, 37 ms of it in
parallel_apply).

Here each replica is a persistent module copy on its device with STATIC
parameter / buffer / input tensors, captured once -- forward and backward
separately -- with ``torch.cuda.make_graphed_callables``.  A step then is:

  forward   pull the device-0 parameters into every replica's static
            parameters (one multi-copy kernel per device, comm_ops.pull_copy),
            copy each input chunk into its static input, replay every
            replica's forward graph (a host call of ~10 us each, no threads),
            gather the outputs onto the output device;
  backward  scatter the output gradient, replay every replica's backward
            graph (one autograd call over all replicas), sum the replicas'
            parameter gradients onto device 0 with the N-way reduce-add
            kernel (comm_ops.reduce_add_coalesced) -- returned as the
            gradient of the real parameters, exactly like ``Replicate``.

Replica 0's buffers ARE the module's buffers (its running statistics are
updated, as upstream); the others' buffers are refreshed from device 0 each
step.  Requirements: training mode, a fixed per-replica batch (a different
batch shape -- e.g. a ragged last batch -- runs the eager path), and a
capture-safe forward (no host synchronisation), which every native op here
is (bench.py --graph captures the same ops).
"""
from __future__ import annotations

import copy
from typing import List, Optional, Sequence

import torch
import torch.nn as nn

# one replay stream per replica (False: every replica on the current stream; A/B)
PER_REPLICA_STREAMS = True

from . import comm_ops
from ..utils.graphs import no_gc_during_capture


def _static_copy(module: nn.Module, device: torch.device, share_buffers_with: Optional[nn.Module]) -> nn.Module:
    rep = copy.deepcopy(module).to(device)
    for p in rep.parameters():
        p.grad = None
        p.requires_grad_(True)
    if share_buffers_with is not None:
        src = dict(share_buffers_with.named_buffers())
        for name, _ in list(rep.named_buffers()):
            mod = rep
            *path, leaf = name.split(".")
            for k in path:
                mod = getattr(mod, k)
            mod._buffers[leaf] = src[name]
    return rep


def check_replica_layout(devices: Sequence[torch.device], stream_devices: Sequence[torch.device],
                         stream_ids: Sequence[int], tensor_devices: Sequence[Sequence[torch.device]],
                         per_replica_streams: bool = True) -> None:
    """The invariants a captured replica set relies on:
    replica i's stream lives on replica i's device; with per-replica streams no
    two replicas share one (a shared stream would serialise replicas and, on
    distinct devices, replay a graph on a foreign device's queue); every static
    parameter / buffer / input of replica i is on device i.  (Each replica is
    captured by its own make_graphed_callables call, which gives it its own
    graph memory pool.)  Raises RuntimeError naming the first violation."""
    if not (len(devices) == len(stream_devices) == len(stream_ids) == len(tensor_devices)):
        raise RuntimeError("GraphedReplicas: one stream and one tensor set per replica")
    for i, (d, sd) in enumerate(zip(devices, stream_devices)):
        if torch.device(sd) != torch.device(d):
            raise RuntimeError(f"GraphedReplicas: replica {i}'s stream is on {sd}, the replica on {d}")
        bad = [t for t in tensor_devices[i] if torch.device(t) != torch.device(d)]
        if bad:
            raise RuntimeError(f"GraphedReplicas: replica {i} (device {d}) holds a static tensor on {bad[0]}")
    if per_replica_streams and len(set(zip(map(str, stream_devices), stream_ids))) != len(stream_ids):
        raise RuntimeError("GraphedReplicas: two replicas share a replay stream")


class GraphedReplicas:
    """Per-device static replicas of ``module`` with captured forward and
    backward graphs, for one per-replica input shape."""

    def __init__(self, module: nn.Module, devices: Sequence[torch.device], chunk: torch.Tensor):
        self.module = module
        self.devices = [torch.device(d) for d in devices]
        self.params = [p for p in module.parameters()]
        self.buffers = [b for b in module.buffers()]
        self.shape, self.dtype = tuple(chunk.shape), chunk.dtype
        self.cl = chunk.dim() == 4 and chunk.is_contiguous(memory_format=torch.channels_last)
        self.replicas: List[nn.Module] = []
        self.inputs: List[torch.Tensor] = []
        for i, d in enumerate(self.devices):
            rep = _static_copy(module, d, module if i == 0 else None)
            self.replicas.append(rep)
            x = torch.empty(self.shape, dtype=self.dtype, device=d,
                            memory_format=torch.channels_last if self.cl else torch.contiguous_format)
            x.copy_(chunk)
            self.inputs.append(x)
        self.rparams = [list(r.parameters()) for r in self.replicas]
        # one stream per replica: replicas sharing a device replay concurrently
        # (a 64-image ResNet-50 pass leaves most of an MI355X idle); autograd
        # runs each replica's backward graph on the stream its forward used
        # (PER_REPLICA_STREAMS = False: replay everything on the current stream)
        if PER_REPLICA_STREAMS:
            self.streams = [torch.cuda.Stream(device=d) for d in self.devices]
        else:
            self.streams = [torch.cuda.current_stream(d) for d in self.devices]
        self.rbuffers = [list(r.buffers()) for r in self.replicas]
        check_replica_layout(self.devices, [s.device for s in self.streams], [s.stream_id for s in self.streams],
                             [[t.device for t in (self.rparams[i] + self.rbuffers[i] + [self.inputs[i]])]
                              for i in range(len(self.devices))], PER_REPLICA_STREAMS)
        self.graphed = []
        # the capture's warm-up iterations run replica 0 for real: keep the
        # module's running statistics as they were (its buffers are shared)
        saved = [b.detach().clone() for b in self.buffers]
        # no Python garbage collection inside the captures (utils/graphs.py)
        with no_gc_during_capture():
            for rep, x, d in zip(self.replicas, self.inputs, self.devices):
                with torch.cuda.device(d):
                    self.graphed.append(torch.cuda.make_graphed_callables(rep, (x,)))
        with torch.no_grad():
            for b, v in zip(self.buffers, saved):
                b.copy_(v)

    def matches(self, chunks: Sequence[torch.Tensor]) -> bool:
        return len(chunks) == len(self.devices) and all(
            tuple(c.shape) == self.shape and c.dtype == self.dtype for c in chunks)

    def refresh(self) -> None:
        """Device-0 parameters (and, for replicas >= 1, buffers) -> the static copies."""
        with torch.no_grad():
            for i, d in enumerate(self.devices):
                srcs = [p.detach() for p in self.params]
                dsts = [p.detach() for p in self.rparams[i]]
                if i > 0:
                    srcs += [b for b in self.buffers]
                    dsts += self.rbuffers[i]
                with torch.cuda.device(d):
                    comm_ops.pull_copy(srcs, dsts)


class _GraphedDPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gr: GraphedReplicas, output_device, chunks, *params):
        gr.refresh()
        with torch.no_grad():
            for x, c in zip(gr.inputs, chunks):
                x.copy_(c, non_blocking=True)
        mains = {d: torch.cuda.current_stream(d) for d in gr.devices}
        outs = []
        with torch.enable_grad():
            for g, x, d, st in zip(gr.graphed, gr.inputs, gr.devices, gr.streams):
                st.wait_stream(mains[d])  # refreshed parameters and copied inputs
                with torch.cuda.stream(st):
                    outs.append(g(x))
        for d, st in zip(gr.devices, gr.streams):
            mains[d].wait_stream(st)
        ctx.gr, ctx.outs = gr, outs
        ctx.sizes = [o.shape[0] for o in outs]
        return comm_ops.gather_tensors([o.detach() for o in outs], output_device, 0)

    @staticmethod
    def backward(ctx, g):
        gr = ctx.gr
        parts = comm_ops.scatter_tensor(g.contiguous(), gr.devices, 0, ctx.sizes)
        torch.autograd.backward(ctx.outs, parts)
        per_dev = []
        for ps in gr.rparams:
            per_dev.append([p.grad if p.grad is not None else torch.zeros_like(p) for p in ps])
        red = comm_ops.reduce_add_coalesced(per_dev, gr.devices[0])
        for ps in gr.rparams:
            for p in ps:
                p.grad = None
        ctx.outs = None
        return (None, None, None) + tuple(red)


def graphed_forward(gr: GraphedReplicas, chunks: Sequence[torch.Tensor], output_device) -> torch.Tensor:
    return _GraphedDPFn.apply(gr, output_device, list(chunks), *gr.params)
