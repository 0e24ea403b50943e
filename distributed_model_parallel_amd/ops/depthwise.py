"""3x3 depthwise convolution on channels-last tensors (``csrc/conv/depthwise.hip``).

:class:`DepthwiseConv2d` is a drop-in ``nn.Conv2d(C, C, 3, stride, 1,
groups=C, bias=False)`` (same parameter, same state_dict key) that takes the
native forward / data-grad / weight-grad kernels on MI355X when the input is
channels-last with C a multiple of the vector width, and PyTorch's conv
otherwise (CPU, odd shapes)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0}


def _native_ok(x: torch.Tensor) -> bool:
    if not _native.gpu_path(x):
        return False
    vec = 8 if x.dtype == torch.bfloat16 else 4
    return (x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 4 and x.shape[1] % vec == 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


class _DWConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, moments=False):
        C = _native.require("depthwise conv")
        y, mom = C.dwconv3x3_forward(x, w, stride, moments)
        ctx.save_for_backward(x, w)
        ctx.stride = stride
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        # the moments output never gets a gradient: do not let autograd build a
        # zero [2C+1] fp64 tensor for it every backward (one fill launch per layer)
        ctx.set_materialize_grads(False)
        return y, mom

    @staticmethod
    def backward(ctx, dy, _dmom=None):
        if dy is None:
            return None, None, None, None
        x, w = ctx.saved_tensors
        C = _native.require("depthwise conv backward")
        dy = dy.contiguous(memory_format=torch.channels_last).to(x.dtype)
        dx = C.dwconv3x3_dgrad(dy, w, ctx.stride, x.shape[2], x.shape[3]) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            from . import grad_accum, wgrad_stream
            acc = grad_accum.target(w)  # micro-batch accumulation: the column reduce adds into w.grad
            with wgrad_stream.side(w, dy, x):  # beside the data-gradient chain
                dw = C.dwconv3x3_wgrad(dy, x, ctx.stride, w.dtype, out=acc)
            if acc is not None:
                dw = None
        return dx, dw, None, None


def depthwise_conv3x3(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, moments: bool = False):
    """Returns y, or (y, moments-or-None) when `moments` is requested."""
    if _native_ok(x) and stride in (1, 2):
        _STATS["native"] += 1
        y, mom = _DWConvFn.apply(x, weight, stride, moments)
        return (y, mom) if moments else y
    _STATS["torch"] += 1
    y = F.conv2d(x, weight, None, stride, 1, 1, x.shape[1])
    return (y, None) if moments else y


class DepthwiseConv2d(nn.Conv2d):
    def __init__(self, channels: int, stride: int = 1, device=None, dtype=None):
        super().__init__(channels, channels, 3, stride=stride, padding=1, groups=channels, bias=False,
                         device=device, dtype=dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return depthwise_conv3x3(x, self.weight, self.stride[0])

    def forward_with_moments(self, x: torch.Tensor):
        return depthwise_conv3x3(x, self.weight, self.stride[0], moments=True)
