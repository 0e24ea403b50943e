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
    def forward(ctx, logits, target, ignore_index, scale, acc):
        C = _native.require("cross_entropy")
        loss, lse, stats = C.cross_entropy_fwd(logits, target, ignore_index, scale, acc)
        ctx.save_for_backward(logits, target, lse, stats)
        ctx.ignore_index = ignore_index
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, stats = ctx.saved_tensors
        C = _native.require("cross_entropy backward")
        dx = C.cross_entropy_bwd(g.reshape(1), logits, target, lse, stats, ctx.ignore_index)
        return dx, None, None, None, None


def _native_ce_ok(logits: torch.Tensor, target: torch.Tensor) -> bool:
    return (_native.gpu_path(logits) and logits.dim() == 2 and logits.dtype in (torch.float32, torch.bfloat16)
            and logits.stride(1) == 1 and target.dtype == torch.int64 and target.dim() == 1)


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy in fp32 (same value as F.cross_entropy(logits.float(), target))."""
    if _native_ce_ok(logits, target):
        _STATS["native"] += 1
        return _CrossEntropyFn.apply(logits, target.contiguous(), int(ignore_index), 1.0, None)
    _STATS["torch"] += 1
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)


def cross_entropy_with_stats(logits: torch.Tensor, target: torch.Tensor, scale: float,
                             stats: torch.Tensor) -> torch.Tensor:
    """``scale * cross_entropy(logits, target)``, and ``stats`` (fp64 [3]) +=
    (that loss, top-1 correct, top-min(5, C) correct) -- a pipeline micro-batch's
    loss and statistics.  Native: the two cross-entropy kernels also rank the
    target among the logits (no fp32 copy of the logits, no topk / sort and
    statistics kernels); otherwise the PyTorch composition."""
    if _native_ce_ok(logits, target) and stats.is_cuda and stats.dtype == torch.float64 \
            and stats.numel() == 3 and stats.is_contiguous():
        _STATS["native"] += 1
        return _CrossEntropyFn.apply(logits, target.contiguous(), -100, float(scale), stats)
    _STATS["torch"] += 1
    lf = logits.float()
    loss = F.cross_entropy(lf, target) * scale
    with torch.no_grad():
        maxk = min(5, lf.shape[1])
        pred = lf.topk(maxk, 1, True, True).indices.t()
        correct = pred.eq(target.view(1, -1))
        stats[0] += loss.detach().double()
        stats[1] += correct[:1].sum().double()
        stats[2] += correct[:maxk].sum().double()
    return loss
