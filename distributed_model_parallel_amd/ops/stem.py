"""ResNet stem convolution (7x7, stride 2, pad 3, 3 -> C channels) on the MFMA
implicit GEMM via space-to-depth (``csrc/conv/stem.hip``).

The 3-channel input cannot feed 64-deep K tiles directly (MIOpen runs this
conv at ~140 TF/s).  Space-to-depth by 2 turns it into a 4x4 / stride-1 conv
on 12 channels (padded to 16); four adjacent 16-channel pixels form one
64-channel "row tap" (``conv_nt(..., kc=64)``), so the whole stem is one
M x C x 256 implicit GEMM -- with the BN moments of its output in the
epilogue -- and its weight gradient the matching split-M TN GEMM.  The
7x7 -> 4x4x16 weight re-layout is a few differentiable torch ops on the
64x3x7x7 weight, so autograd folds the gradient back for free.

The input image needs no gradient; an input that requires one (or anything
the kernels do not cover) takes ``F.conv2d``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0, "halo": 0}
# 224-px inputs (Wo = 112): the persistent halo-tiled stem kernels
# (csrc/conv/stem_halo.hip) instead of the generic row-tap implicit GEMM;
# DMP_DISABLE=stem_halo for A/B runs.
_HALO = not _native.disabled("stem_halo")


def stem_wmat(w: torch.Tensor) -> torch.Tensor:
    """[Cout, 3, 7, 7] -> [Cout, 4 * 64]: K index = r*64 + q*16 + (dy*2+dx)*3 + c holds
    W[c, 2r+dy, 2q+dx] (zero where 2r+dy or 2q+dx is 7, and for channels 12..15)."""
    co = w.shape[0]
    wp = F.pad(w.contiguous(), (0, 1, 0, 1))                      # [co, 3, 8, 8]
    wp = wp.view(co, 3, 4, 2, 4, 2).permute(0, 2, 4, 3, 5, 1)     # co, r, q, dy, dx, c
    wp = F.pad(wp.reshape(co, 4, 4, 12), (0, 4))                  # 16 channels per s2d pixel
    return wp.reshape(co, 256).contiguous()


class _StemFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wmat, moments):
        C = _native.require("stem conv")
        n, _, h, w = x.shape
        ho, wo = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
        s = C.space_to_depth2(x, 3)                                # [n, 16, (h+7)//2, (w+7)//2]
        halo = _HALO and C.stem_halo_supported(s.shape[2], s.shape[3], ho, wo)
        if halo:  # halo-tiled kernel, weights in VGPRs (csrc/conv/stem_halo.hip)
            _STATS["halo"] += 1
            y2, mom = C.stem_halo_fwd(s, wmat.contiguous(), ho, moments)
            if not moments:
                mom = None
        else:
            y2, mom = C.conv_nt(s, wmat, 4, 1, 1, 0, ho, wo, mode="moments" if moments else "store", kc=64)
        ctx.save_for_backward(s)
        ctx.geo = (n, ho, wo, wmat.dtype, halo)
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        ctx.set_materialize_grads(False)
        return y2.view(n, ho, wo, -1).permute(0, 3, 1, 2), mom

    @staticmethod
    def backward(ctx, dy, _dmom):
        if dy is None:
            return None, None, None
        (s,) = ctx.saved_tensors
        n, ho, wo, wdt, halo = ctx.geo
        C = _native.require("stem conv backward")
        dy2 = dy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(n * ho * wo, -1)
        if halo:
            dw = C.stem_halo_wgrad(dy2.to(s.dtype), s, ho, wdt)
        else:
            dw = C.conv_wgrad(dy2.to(s.dtype), s, 4, 1, 1, 0, ho, wo, wdt, kc=64)
        return None, dw, None


def _native_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    return (_native.gpu_path(x) and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape[1] == 3 and x.is_contiguous(memory_format=torch.channels_last)
            and not x.requires_grad and conv.kernel_size == (7, 7) and conv.stride == (2, 2)
            and conv.padding == (3, 3) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.bias is None)


class StemConv2d(nn.Conv2d):
    """Drop-in ``nn.Conv2d(3, cout, 7, stride=2, padding=3, bias=False)``."""

    def __init__(self, cin: int = 3, cout: int = 64, device=None, dtype=None):
        super().__init__(cin, cout, 7, stride=2, padding=3, bias=False, device=device, dtype=dtype)

    def forward_with_moments(self, x: torch.Tensor):
        if _native_ok(self, x):
            _STATS["native"] += 1
            y, mom = _StemFn.apply(x, stem_wmat(self.weight), True)
            return y, mom
        _STATS["torch"] += 1
        return super().forward(x), None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _native_ok(self, x):
            _STATS["native"] += 1
            return _StemFn.apply(x, stem_wmat(self.weight), False)[0]
        _STATS["torch"] += 1
        return super().forward(x)


# --------------------------------------------------------------------------- #
# Stride-1 few-channel conv (MobileNetV2 CIFAR stem: 3x3, pad 1, 3 -> 32)
# --------------------------------------------------------------------------- #
def rowtap_wmat(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin<=16, k, k] -> [Cout, k * 64]: row r holds 4 pixels x 16 channels;
    pixels q >= k and channels >= Cin carry zero weights."""
    co, ci, k, _ = w.shape
    wp = w.contiguous().permute(0, 2, 3, 1)                         # co, r, q, c
    wp = F.pad(wp, (0, 16 - ci, 0, 4 - k))                          # [co, k, 4, 16]
    return wp.reshape(co, k * 64).contiguous()


class _RowTapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wmat, k, pad, moments):
        C = _native.require("row-tap conv")
        n, _, h, w = x.shape
        xp = C.pad_channels16(x, pad, 4 - k)                         # [n, 16, h+2p, w+2p+4-k]
        y2, mom = C.conv_nt(xp, wmat, k, 1, 1, 0, h, w, mode="moments" if moments else "store", kc=64)
        ctx.save_for_backward(xp)
        ctx.geo = (n, h, w, k, wmat.dtype)
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        ctx.set_materialize_grads(False)
        return y2.view(n, h, w, -1).permute(0, 3, 1, 2), mom

    @staticmethod
    def backward(ctx, dy, _dmom):
        if dy is None:
            return None, None, None, None, None
        (xp,) = ctx.saved_tensors
        n, h, w, k, wdt = ctx.geo
        C = _native.require("row-tap conv backward")
        dy2 = dy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1).reshape(n * h * w, -1)
        dw = C.conv_wgrad(dy2.to(xp.dtype), xp, k, 1, 1, 0, h, w, wdt, kc=64)
        return None, dw, None, None, None


_ROWTAP = not _native.disabled("rowtap_stem")


def _rowtap_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    k = conv.kernel_size[0]
    return (_ROWTAP and _native.gpu_path(x) and x.dtype == torch.bfloat16 and conv.weight.dtype == torch.bfloat16
            and x.dim() == 4 and x.shape[1] <= 16 and x.is_contiguous(memory_format=torch.channels_last)
            and not x.requires_grad and conv.kernel_size == (k, k) and k <= 4 and conv.stride == (1, 1)
            and conv.padding == (k // 2, k // 2) and k % 2 == 1 and conv.dilation == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.out_channels % 8 == 0)


class RowTapConv2d(nn.Conv2d):
    """Drop-in ``nn.Conv2d(cin <= 16, cout, k <= 3 odd, stride=1, padding=k//2, bias=False)``
    on the MFMA implicit GEMM: the input is zero-padded to 16 channels and each
    kernel row becomes one 64-channel row tap (4 adjacent pixels, the 4th with
    zero weights)."""

    def __init__(self, cin: int, cout: int, kernel_size: int = 3, device=None, dtype=None):
        super().__init__(cin, cout, kernel_size, stride=1, padding=kernel_size // 2, bias=False,
                         device=device, dtype=dtype)

    def forward_with_moments(self, x: torch.Tensor):
        if _rowtap_ok(self, x):
            _STATS["native"] += 1
            y, mom = _RowTapFn.apply(x, rowtap_wmat(self.weight), self.kernel_size[0], self.padding[0], True)
            return y, mom
        _STATS["torch"] += 1
        return super().forward(x), None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if _rowtap_ok(self, x):
            _STATS["native"] += 1
            return _RowTapFn.apply(x, rowtap_wmat(self.weight), self.kernel_size[0], self.padding[0], False)[0]
        _STATS["torch"] += 1
        return super().forward(x)
