"""Linear layers for the ViT encoder with native backward side passes
(``csrc/linear/bias_act.hip``).

* ``Linear``: drop-in ``nn.Linear``.  Forward is one library GEMM with the bias
  in its epilogue (``addmm`` -> hipBLASLt ``Bias`` kernels).  Backward runs the
  two library GEMMs (dx, dW) and takes the bias gradient with our column-sum
  kernel instead of PyTorch's generic reduce (1.77 ms -> see
  ``profiles/vit_b16_bs128_1gpu_v3.md``).
* ``linear_gelu``: fc1 + exact GELU; the backward fuses gelu'(h) with fc1's
  bias gradient in one pass over the pre-activation.

CPU tensors, non-bf16 dtypes and widths that are not a multiple of 256 use
the plain PyTorch ops (same math)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0}


def _native_ok(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> bool:
    if not _native.gpu_path(x):
        return False
    C = _native.native()
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and b is not None
            and b.dtype == torch.bfloat16 and C.colsum_supported(w.shape[0]))


def _weight_grads(ctx, dy2, x2, w):
    dx = dy2.mm(w) if ctx.needs_input_grad[0] else None
    dw = dy2.t().mm(x2) if ctx.needs_input_grad[1] else None
    return dx, dw


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        y = torch.addmm(b, x2, w.t())
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        C = _native.require("linear backward")
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx, dw = _weight_grads(ctx, dy2, x2, w)
        db = C.bias_grad(dy2, w.dtype) if ctx.needs_input_grad[2] else None
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db


class _LinearGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        h = torch.addmm(b, x2, w.t())
        ctx.save_for_backward(x2, w, h)
        ctx.xshape = x.shape
        return F.gelu(h).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, da):
        x2, w, h = ctx.saved_tensors
        C = _native.require("linear+gelu backward")
        dh, db = C.gelu_bwd_bias_grad(da.reshape(h.shape).contiguous(), h, w.dtype)
        dx, dw = _weight_grads(ctx, dh, x2, w)
        return (dx.view(ctx.xshape) if dx is not None else None), dw, \
            (db if ctx.needs_input_grad[2] else None)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    if _native_ok(x, weight, bias):
        _STATS["native"] += 1
        return _LinearFn.apply(x, weight, bias)
    _STATS["torch"] += 1
    return F.linear(x, weight, bias)


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """gelu(x @ W^T + b) (exact erf GELU, as ``nn.GELU()``)."""
    if _native_ok(x, weight, bias):
        _STATS["native"] += 1
        return _LinearGeluFn.apply(x, weight, bias)
    _STATS["torch"] += 1
    return F.gelu(F.linear(x, weight, bias))


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` whose backward uses the native bias-gradient kernel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)
