"""Fused softmax cross-entropy (``csrc/loss/cross_entropy.hip``).

``cross_entropy(logits, target)`` == ``F.cross_entropy(logits.float(), target)``
(mean reduction, ``ignore_index``), computed in fp32 from bf16 or fp32 logits
without materialising an fp32 copy: one forward kernel (row max, exp-sum, loss,
saved log-sum-exp) plus a one-block mean, and one backward kernel writing
d(logits) in the logits' dtype.  Reference criterion: ``nn.CrossEntropyLoss``
(``model_parallel.py:106,147``, ``data_parallel.py:89``).
CPU tensors and other shapes use ``F.cross_entropy``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0}


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        C = _native.require("cross_entropy")
        loss, lse, stats = C.cross_entropy_fwd(logits, target, ignore_index)
        ctx.save_for_backward(logits, target, lse, stats)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, stats = ctx.saved_tensors
        C = _native.require("cross_entropy backward")
        dx = C.cross_entropy_bwd(g.reshape(1), logits, target, lse, stats, ctx.ignore_index)
        return dx, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy in fp32 (same value as F.cross_entropy(logits.float(), target))."""
    if (_native.gpu_path(logits) and logits.dim() == 2 and logits.dtype in (torch.float32, torch.bfloat16)
            and logits.stride(1) == 1 and target.dtype == torch.int64 and target.dim() == 1):
        _STATS["native"] += 1
        return _CrossEntropyFn.apply(logits, target.contiguous(), int(ignore_index))
    _STATS["torch"] += 1
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
