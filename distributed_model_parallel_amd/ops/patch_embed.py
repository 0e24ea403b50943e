"""ViT patch embedding (a p x p / stride-p convolution) as one MFMA GEMM.

With stride == kernel the convolution has no overlap: it is exactly a GEMM of
the non-overlapping patches [B * (H/p) * (W/p), p * p * C] with the weight
viewed as [D, p * p * C].  Forward: one patchify copy of the image (the only
pass over it) and ``gemm_xl`` with the bias in its store; backward: the
weight gradient dy^T @ patches on the TN ping-pong kernel and the bias
gradient as a column sum -- no MIOpen ``igemm_fwd`` / ``igemm_wrw``
(0.41 ms of the ViT-B/16 step).  The patch vector is ordered
(kh, kw, c) so the copy reads a channels-last image in 3-element runs and
writes rows contiguously; the weight is permuted to match (a 1.2 MB copy).

Capability: the torchvision ``conv_proj`` of ViT-B/16 (parameter layout
[D, C, p, p] kept, so state dicts stay compatible); design: ours.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0}


def _patchify(x: torch.Tensor, p: int) -> torch.Tensor:
    b, c, h, w = x.shape
    t = x.reshape(b, c, h // p, p, w // p, p).permute(0, 2, 4, 3, 5, 1)  # [B, h/p, w/p, p, p, C]
    return t.reshape(b * (h // p) * (w // p), p * p * c)


def _wmat(weight: torch.Tensor) -> torch.Tensor:
    d = weight.shape[0]
    return weight.permute(0, 2, 3, 1).reshape(d, -1).contiguous()  # [D, (kh, kw, c)]


class _PatchEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, p):
        C = _native.require("patch embed")
        b, c, h, w = x.shape
        patches = _patchify(x, p)
        y = C.gemm_xl(patches, _wmat(weight), "bias", bias=bias)
        ctx.save_for_backward(patches, weight)
        ctx.geom = (b, c, h, w, p)
        return y.view(b, (h // p) * (w // p), weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from .linear import _wgrad
        C = _native.require("patch embed backward")
        patches, weight = ctx.saved_tensors
        b, c, h, w, p = ctx.geom
        d = weight.shape[0]
        dy2 = dy.reshape(-1, d).contiguous()
        dw = db = dx = None
        if ctx.needs_input_grad[1]:
            from . import wgrad_stream
            with wgrad_stream.side(weight, dy2, patches):  # the layout copy follows the GEMM on S
                dwm = _wgrad(dy2, patches, weight)  # [D, (kh, kw, c)]
                dw = dwm.view(d, p, p, c).permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last) \
                    if weight.is_contiguous(memory_format=torch.channels_last) else \
                    dwm.view(d, p, p, c).permute(0, 3, 1, 2).contiguous()
        if ctx.needs_input_grad[2]:
            db = C.bias_grad(dy2, weight.dtype)
        if ctx.needs_input_grad[0]:  # the image rarely needs a gradient: plain GEMM + un-patchify
            dp = dy2.mm(_wmat(weight)).view(b, h // p, w // p, p, p, c)
            dx = dp.permute(0, 5, 1, 3, 2, 4).reshape(b, c, h, w)
        return dx, dw, db, None


class PatchEmbed(nn.Conv2d):
    """Drop-in ``nn.Conv2d(C, D, p, stride=p)`` returning tokens [B, T, D]
    (the conv output flattened and transposed, as ViT consumes it)."""

    def __init__(self, in_channels: int, dim: int, patch: int):
        super().__init__(in_channels, dim, patch, stride=patch)

    def _native_ok(self, x: torch.Tensor) -> bool:
        p = self.kernel_size[0]
        b, c, h, w = x.shape
        if not (_native.gpu_path(x) and x.dtype == torch.bfloat16 and self.weight.dtype == torch.bfloat16
                and self.bias is not None and self.bias.dtype == torch.bfloat16):
            return False
        from .linear import _XL, _XL_MIN_ROWS
        C = _native.native()
        return (_XL and h % p == 0 and w % p == 0 and b * (h // p) * (w // p) >= _XL_MIN_ROWS
                and (p * p * c) % 64 == 0 and self.weight.shape[0] % 64 == 0
                and C.colsum_supported(self.weight.shape[0]))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self._native_ok(x):
            _STATS["native"] += 1
            return _PatchEmbedFn.apply(x, self.weight, self.bias, self.kernel_size[0])
        _STATS["torch"] += 1
        return F.conv2d(x, self.weight, self.bias, self.stride).flatten(2).transpose(1, 2)
