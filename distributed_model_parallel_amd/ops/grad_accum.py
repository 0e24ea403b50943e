"""Parameter gradients accumulated by the producing kernels (micro-batch
gradient accumulation without the autograd engine's adds).

A pipeline stage runs M micro-batches per step and sums their parameter
gradients.  Through autograd every micro-batch's weight gradient is a fresh
tensor that AccumulateGrad then adds into ``p.grad``: one elementwise add per
parameter per micro-batch (MobileNetV2: ~170 per 64-image micro-batch, plus
dtype copies), each a few microseconds of a launch-bound step.  Inside
:func:`accumulate_param_grads` the native ops instead hand ``p.grad`` to their
weight-gradient kernels, which ADD their result into it in the pass that
already writes the gradient (the split-K reduce of the MFMA weight-gradient
GEMMs, the depthwise column reduce, the BN backward's affine gradients), and
return None to autograd for that parameter, so no AccumulateGrad runs.

Rules (checked by :func:`target`): the mode is on, the parameter's ``grad``
exists (the caller zeroes it before the first micro-batch), has the
parameter's dtype, shape and a dense layout.  Otherwise the op returns its
gradient as usual.  Nothing that hooks AccumulateGrad (DDP's reducer) may run
inside the mode: the pipeline enables it for its stage module only, which DDP
never wraps.

Capability: the reference's micro-batch gradient accumulation is PyTorch's
(``model_parallel.py:99-157`` backward per micro-batch into ``.grad``); the
in-kernel form is ours.
"""
from __future__ import annotations

import contextlib
from typing import Iterator, Optional

import torch

_ON = [False]
_STATS = {"kernel": 0}


@contextlib.contextmanager
def accumulate_param_grads(enabled: bool = True) -> Iterator[None]:
    prev = _ON[0]
    _ON[0] = bool(enabled)
    try:
        yield
    finally:
        _ON[0] = prev


def active() -> bool:
    return _ON[0]


def target(p: Optional[torch.Tensor], channels_last_ok: bool = True) -> Optional[torch.Tensor]:
    """``p.grad`` when the producing kernel may add into it, else None."""
    if not _ON[0] or p is None or not p.requires_grad:
        return None
    g = p.grad
    if g is None or g.dtype != p.dtype or g.shape != p.shape or not g.is_cuda:
        return None
    if not (g.is_contiguous() or (channels_last_ok and g.dim() == 4
                                  and g.is_contiguous(memory_format=torch.channels_last))):
        return None
    if g.data_ptr() % 16:
        return None
    _STATS["kernel"] += 1
    return g


def stats() -> dict:
    return dict(_STATS)
