"""SyncBatchNorm: batch statistics over all ranks with ONE RCCL all-reduce of
the fp64 moments [sum x, sum x^2, rows] per layer forward and one all-reduce of
[sum dz, sum dz*(x-mean)] per layer backward.

Parity: upstream SyncBatchNorm as "prepared for" by DDP's init helper
(reference Readme.md:151).  Upstream all-gathers per-rank
mean/invstd/count and combines them; here the moments are additive, so a single
in-place all-reduce (north star: "SyncBatchNorm as an RCCL all-reduce of
mean/var") replaces gather + combine, and the global row count rides in the
same buffer so no host synchronisation is needed.  The kernels are the fused
channels-last BN(+residual)(+ReLU) ones of :mod:`..ops.batchnorm`.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..comm.rccl import Communicator, verify_comm_layout
from ..ops.batchnorm import BatchNormAct2d
from ..utils.env import single_rank_comm

# One communicator per (device, group) shared by every SyncBatchNorm layer and
# never by DDP: the moment all-reduces are enqueued on the COMPUTE stream, the
# DDP bucket all-reduces on the reducer's side stream -- two streams driving one
# ncclComm would serialise the ~100 tiny per-step SyncBN collectives behind
# (and interleave them with) the 25 MB bucket collectives.
#
# Ordering (why two communicators on two streams cannot deadlock across ranks):
# an RCCL kernel blocks its stream -- and, when GPU_MAX_HW_QUEUES (4 here) makes
# two streams share a hardware queue, everything queued behind it -- until
# every peer has launched the matching kernel.  A cross-communicator deadlock
# needs two ranks to submit the SyncBN and bucket collectives in DIFFERENT
# interleavings.  They cannot: (1) each communicator's own sequence is the same
# on every rank (SyncBN: layer order of the shared module; DDP: buckets
# launched strictly in index order, reducer.cpp launch_ready_prefix_locked);
# (2) both are enqueued from ONE host thread per rank -- the forward thread
# for the forward moments, the autograd device thread for the SyncBN backward
# nodes and for the post-accumulate hooks that launch buckets -- in an order
# fixed by the autograd graph, which is identical on every rank (bucket
# rebuilds follow rank 0's recorded order).  So the merged submission order is
# rank-independent and every blocking kernel waits only for kernels its peers
# submitted before theirs.  tests/test_comm_ordering.py records the merged
# order on every rank of a DDP + SyncBN ResNet-18 and requires it identical.
# Which streams share a hardware queue follows stream creation order; that the
# communicators (and so their streams) were created in the same order with the
# same flags on every rank is not assumed but checked collectively when this
# communicator is created (comm/rccl.py verify_comm_layout).
_COMMS = {}


def syncbn_communicator(device: torch.device, group: Optional[dist.ProcessGroup] = None) -> Communicator:
    key = (str(device), id(group) if group is not None else None)
    if key not in _COMMS:
        _COMMS[key] = Communicator(device, group, purpose="syncbn")
        # the second stream-driving communicator exists now: every rank must
        # have created the same ones in the same order (comm/rccl.py _LAYOUT)
        verify_comm_layout("SyncBatchNorm communicator", group)
    return _COMMS[key]


def reset_syncbn_communicators() -> None:
    _COMMS.clear()


class SyncBatchNorm(BatchNormAct2d):
    def __init__(self, num_features: int, eps: float = 1e-5, momentum: Optional[float] = 0.1,
                 affine: bool = True, track_running_stats: bool = True,
                 process_group: Optional[dist.ProcessGroup] = None, act: Optional[str] = None,
                 device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, act,
                         device, dtype)
        self.process_group = process_group
        self._comm: Optional[Communicator] = None

    def _communicator(self, device: torch.device) -> Communicator:
        if self._comm is None:
            self._comm = syncbn_communicator(device, self.process_group)
        return self._comm

    def _moment_reducers(self):
        if not (dist.is_available() and dist.is_initialized()):
            return None, None
        if dist.get_world_size(self.process_group) == 1 and not single_rank_comm():
            return None, None  # the all-reduce of one rank's moments is the identity
        dev = self.weight.device if self.weight is not None else self.running_mean.device
        comm = self._communicator(dev)

        def reduce(t: torch.Tensor) -> torch.Tensor:
            # tiny ([2C+1] fp64) and needed by the very next kernel: enqueue on the
            # compute stream itself (no side stream / event pair per layer)
            t = t.contiguous()
            comm.all_reduce(t, "sum", on_current_stream=True)
            return t

        return reduce, reduce

    @classmethod
    def convert_sync_batchnorm(cls, module: nn.Module,
                               process_group: Optional[dist.ProcessGroup] = None) -> nn.Module:
        """Recursively replace every BatchNorm*d (ours or torch's) by SyncBatchNorm."""
        out = module
        if isinstance(module, nn.modules.batchnorm._BatchNorm) and not isinstance(module, cls):
            out = cls(module.num_features, module.eps, module.momentum, module.affine,
                      module.track_running_stats, process_group,
                      act=getattr(module, "act", None))
            if module.affine:
                with torch.no_grad():
                    out.weight = module.weight
                    out.bias = module.bias
            out.running_mean = module.running_mean
            out.running_var = module.running_var
            out.num_batches_tracked = module.num_batches_tracked
            out.training = module.training
        for name, child in module.named_children():
            out.add_module(name, cls.convert_sync_batchnorm(child, process_group))
        return out
