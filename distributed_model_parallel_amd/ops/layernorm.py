"""LayerNorm over the last dimension on our HIP kernels (``csrc/norm/layernorm.hip``):
one wave per row, x read once per pass, dgamma/dbeta reduced per block.  Used
by ViT-B/16 (BASELINE.json config 5); CPU / unsupported sizes run
``F.layer_norm``."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0, "fused_residual_grad": 0}


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, slot):
        C = _native.require("layernorm")
        d = x.shape[-1]
        xc = x.contiguous()
        y, mean, rstd = C.layernorm_forward(xc, weight, bias, d, float(eps))
        ctx.save_for_backward(xc, weight, mean, rstd)
        ctx.has_b = bias is not None
        ctx.slot = slot
        if slot is not None:
            slot.consumer = True  # the residual branch's gradient joins our dx pass
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, rstd = ctx.saved_tensors
        C = _native.require("layernorm backward")
        pdtype = weight.dtype if weight is not None else torch.float32
        extra = ctx.slot.take() if ctx.slot is not None else None
        if extra is not None:
            extra = extra.contiguous().to(x.dtype)
            _STATS["fused_residual_grad"] += 1
        dx, dw, db = C.layernorm_backward(dy.contiguous().to(x.dtype), x, weight, mean, rstd,
                                          x.shape[-1], pdtype, extra)
        return (dx, dw if weight is not None and ctx.needs_input_grad[1] else None,
                db if ctx.has_b and ctx.needs_input_grad[2] else None, None, None)


def layer_norm(x: torch.Tensor, normalized_shape, weight=None, bias=None, eps: float = 1e-5,
               grad_slot=None):
    """grad_slot (ops.fused.GradSlot): add a residual branch's gradient of x into
    this LayerNorm's dx pass instead of a separate add kernel (pre-LN transformer
    blocks: x + f(ln(x)))."""
    d = x.shape[-1]
    ok = (_native.gpu_path(x) and len(tuple(normalized_shape)) == 1 and normalized_shape[0] == d
          and x.dtype in (torch.bfloat16, torch.float32) and d % 8 == 0 and d <= 2048
          and (weight is None or weight.dtype in (torch.bfloat16, torch.float32))
          and (weight is None or bias is None or weight.dtype == bias.dtype))
    if ok:
        _STATS["native"] += 1
        return _LayerNormFn.apply(x, weight, bias, eps, grad_slot)
    _STATS["torch"] += 1
    return F.layer_norm(x, normalized_shape, weight, bias, eps)


class LayerNorm(nn.LayerNorm):
    """Drop-in ``nn.LayerNorm`` (last-dim normalisation) on the native kernels."""

    def forward(self, x: torch.Tensor, grad_slot=None) -> torch.Tensor:
        return layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps, grad_slot)
