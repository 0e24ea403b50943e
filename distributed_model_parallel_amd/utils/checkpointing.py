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
    return getattr(_state, "recompute", False)


@contextlib.contextmanager
def _recompute_ctx():
    prev = in_recompute()
    _state.recompute = True
    try:
        yield
    finally:
        _state.recompute = prev


def _context_fn():
    return contextlib.nullcontext(), _recompute_ctx()


def checkpoint_sequential(seq: nn.Sequential, segments: int, x: torch.Tensor) -> torch.Tensor:
    mods: Sequence[nn.Module] = list(seq)
    if segments <= 1 or not torch.is_grad_enabled():
        return seq(x)
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
