"""Channels-last max pooling on our HIP kernels (``csrc/pool/maxpool.hip``):
byte-sized argmax instead of PyTorch's int64 index tensor and a gather
backward (no atomics, no zero fill).  Used for the ResNet stem pool; anything
the kernel does not cover (CPU, non-channels-last, dilation, ceil_mode) runs
``F.max_pool2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0, "native_gap": 0}


def _pair1(v) -> int:
    if isinstance(v, (tuple, list)):
        assert len(set(v)) == 1, "only square pooling windows are supported natively"
        return int(v[0])
    return int(v)


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        C = _native.require("maxpool2d")
        y, idx = C.maxpool2d_forward(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.geo = (x.shape[2], x.shape[3], k, s, p)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        C = _native.require("maxpool2d backward")
        h, w, k, s, p = ctx.geo
        dy = dy.contiguous(memory_format=torch.channels_last)
        return C.maxpool2d_backward(dy, idx, h, w, k, s, p), None, None, None


def max_pool2d(x: torch.Tensor, kernel_size, stride=None, padding=0) -> torch.Tensor:
    k = _pair1(kernel_size)
    s = _pair1(stride) if stride is not None else k
    p = _pair1(padding)
    vec = 8 if x.dtype == torch.bfloat16 else 4
    if (_native.gpu_path(x) and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)
            and x.shape[1] % vec == 0 and x.is_contiguous(memory_format=torch.channels_last)
            and 2 * p <= k and k * k <= 255):
        _STATS["native"] += 1
        return _MaxPoolFn.apply(x, k, s, p)
    _STATS["torch"] += 1
    return F.max_pool2d(x, k, s, p)


class _GlobalAvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[2], x.shape[3])
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        C = _native.require("global average pool backward")
        return C.global_avgpool_backward(g.contiguous(), *ctx.hw)


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``adaptive_avg_pool2d(x, 1).flatten(1)`` for channels-last activations.

    The backward writes the broadcast gradient channels-last in one vectorised
    kernel instead of returning an expanded view that the preceding layer's
    backward copies (profiles/README.md finding 13)."""
    vec = 8 if x.dtype == torch.bfloat16 else 4
    if (_native.gpu_path(x) and x.dim() == 4 and x.dtype in (torch.bfloat16, torch.float32)
            and x.shape[1] % vec == 0 and x.is_contiguous(memory_format=torch.channels_last)):
        _STATS["native_gap"] += 1
        return _GlobalAvgPoolFn.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


class MaxPool2d(nn.MaxPool2d):
    """Drop-in ``nn.MaxPool2d`` (square window, no dilation, floor mode)."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.dilation not in (1, (1, 1)) or self.ceil_mode or self.return_indices:
            return super().forward(x)
        return max_pool2d(x, self.kernel_size, self.stride, self.padding)
