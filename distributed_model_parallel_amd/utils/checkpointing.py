"""Activation (gradient) checkpointing for large batches (SURVEY.md D12;
reference Readme.md:168,192 trains batch 1024/2048 "with checkpoint").

:func:`checkpoint_sequential` recomputes each segment of an ``nn.Sequential``
in backward (``torch.utils.checkpoint``, non-reentrant).  BatchNorm layers
would update their running statistics twice (forward + recompute); the
recompute context here switches our BN modules to "no running-stat update"
so checkpointed and plain training produce identical running statistics.
Memory is rarely the constraint on a 288 GB MI355X, but the capability is kept.
"""
from __future__ import annotations

import contextlib
import threading
from typing import Sequence

import torch
import torch.nn as nn
from torch.utils.checkpoint import checkpoint

_state = threading.local()


def in_recompute() -> bool:
    """Inside the backward-time recompute of a checkpointed segment."""
    return getattr(_state, "recompute", False)


def in_checkpoint() -> bool:
    """Inside a checkpointed segment, in its first forward OR its recompute.
    The cross-layer fusions (BN fold, conv+BN moments, parked gradients) test
    this, not in_recompute(): the recompute must rebuild exactly the autograd
    graph (and saved tensors) of the first forward, so both take the plain path."""
    return getattr(_state, "ckpt", False)


@contextlib.contextmanager
def _flags(recompute: bool):
    prev = (in_recompute(), in_checkpoint())
    _state.ckpt = True
    _state.recompute = recompute or prev[0]
    try:
        yield
    finally:
        _state.recompute, _state.ckpt = prev


def _context_fn():
    return _flags(False), _flags(True)


def checkpoint_sequential(seq: nn.Sequential, segments: int, x: torch.Tensor) -> torch.Tensor:
    """Run ``seq`` on x recomputing it in backward in ``segments`` pieces
    (1 = the whole sequence as one piece, <= 0 = no checkpointing)."""
    mods: Sequence[nn.Module] = list(seq)
    if segments <= 0 or not torch.is_grad_enabled():
        for m in mods:  # not seq(x): seq may be a CheckpointedSequential (recursion)
            x = m(x)
        return x
    n = len(mods)
    size = (n + segments - 1) // segments

    def run(lo, hi):
        def f(inp):
            for m in mods[lo:hi]:
                inp = m(inp)
            return inp
        return f

    for lo in range(0, n, size):
        hi = min(n, lo + size)
        x = checkpoint(run(lo, hi), x, use_reentrant=False, context_fn=_context_fn)
    return x


class CheckpointedSequential(nn.Sequential):
    def __init__(self, *mods: nn.Module, segments: int = 2):
        super().__init__(*mods)
        self.segments = segments

    def forward(self, x):
        return checkpoint_sequential(self, self.segments, x)


def _trunks(model: nn.Module):
    """The block sequences of the model zoo: MobileNetV2 ``layers``, ViT
    ``blocks``, ResNet ``layer1..layer4``."""
    for name in ("layers", "blocks", "layer1", "layer2", "layer3", "layer4"):
        m = getattr(model, name, None)
        if isinstance(m, nn.Sequential) and len(m) > 1:
            yield m


def enable_activation_checkpointing(model: nn.Module, segments: int) -> int:
    """Recompute the model's block trunk(s) in backward, ``segments`` segments
    in total (split over ResNet's four layers by their length); returns the
    number of checkpointed Sequentials.  The reference's large-batch runs
    ("2048(checkpoint)", Readme.md:168,192) trade this recompute for memory."""
    if segments <= 1:
        return 0
    from ..parallel.distributed import DistributedDataParallel
    if isinstance(model, DistributedDataParallel) or hasattr(model, "module"):
        model = model.module
    trunks = list(_trunks(model))
    total = sum(len(t) for t in trunks) or 1
    for t in trunks:
        t.__class__ = CheckpointedSequential
        t.segments = max(1, round(segments * len(t) / total))  # 1: the trunk as one segment
    return len(trunks)
