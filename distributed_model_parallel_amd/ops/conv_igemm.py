"""kh x kw convolution (ResNet's 3x3s) as an implicit GEMM on our MFMA kernels
(``csrc/conv/gemm_bf16.hip`` ``conv_nt`` / ``conv_wgrad``), optionally
emitting the BatchNorm moments of its output like the 1x1 path.

  forward   y[N*Ho*Wo, Cout] = im2col(x) @ W^T      tap gather in the A staging,
            K = kh*kw*Cin, W read in its channels_last memory [Cout][kh][kw][Cin]
  (backward: per-shape choice between ours and MIOpen -- see _use_native)
  dgrad     dx = "transposed" implicit GEMM over dy with W permuted to
            [Cin][kh][kw][Cout] (no flip; strided convs handled by the
            divisibility test in the gather; strided convs run as one launch per
            stride phase over only the taps that reach it)
  wgrad     dW[Cout, kh*kw*Cin] = dy^T @ im2col(x)   split-M TN kernel with the
            tap gather in its B staging (channels_last weight memory directly)

Native for bf16 channels_last activations with Cin % 64 == 0 and Cout % 64 == 0
(every ResNet 3x3 except the 7x7 stem, which stays on MIOpen); anything else
uses ``F.conv2d``.  The reference uses torchvision's cuDNN convolutions
(torchvision.models.resnet50 in the DDP scripts).
"""
from __future__ import annotations

import contextlib


from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from . import wgrad_stream, wt_cache

_STATS = {"native": 0, "torch": 0}
# DMP_DISABLE=igemm routes these convs to MIOpen (A/B comparisons, debugging)
ENABLED = not _native.disabled("igemm")
# Backward passes that neither the halo kernels nor conv_xl cover run on
# MIOpen: the generic implicit-GEMM backward (conv_nt transposed / conv_wgrad)
# measured slower on every ResNet-50 shape (profiles/raw_r2/roofline_*.log).
# set_generic_backward(True) routes them to it (any shape; tests).
NATIVE_BWD = False  # set_generic_backward(True): A/B of the generic native backward


def set_generic_backward(on: bool) -> None:
    global NATIVE_BWD
    NATIVE_BWD = bool(on)


def _capturing() -> bool:
    """Inside a hipGraph capture (bench --graph, DataParallel(graphs=True)):
    MIOpen is left out of every captured conv.  Its small-map weight gradient
    replays garbage from the second replay on (round 4,
    tools/graph_replay_bisect.py: a bare nn.Conv2d 512 -> 512 on 2 x 2 maps,
    1e36 gradients from step 1; eager runs of the same module agree bitwise),
    so a captured step takes the native forward / backward for every shape."""
    return torch.cuda.is_current_stream_capturing()


# Weight gradients of 3x3 convs the halo kernel does not cover with Cin % 256
# == 0 (layer 4's stride-2 first block; any layer-3/4 shape at small maps) on
# the TN tap-gather kernel (gemm_xl.hip conv_wgrad_xl) instead of MIOpen's
# igemm_wrw, at every size since round 6: its 4-wave form (gemm_tn_w4 with
# the incremental pixel walk) takes the ResNet-50 layer-3/4 3x3 weight
# gradients at batch 2048 in 0.49-0.52 ms against MIOpen's 0.66-0.78
# (tools/pipe_bench.py --only 3x3wg --lib; the round-4 ping-pong form lost
# above ~50k rows: 0.908 vs 0.655 ms, profiles/raw_r4/wgrad_s2_r4o.md).
_XL_WGRAD = not _native.disabled("xl_conv3")
_STATS["xl_wgrad"] = 0


def _xl_wgrad_ok(cin: int, kh: int, kw: int, rows: int) -> bool:
    return _XL_WGRAD and cin % 256 == 0 and kh == kw and kh > 1

# 256x256 ping-pong implicit GEMM (csrc/gemm/gemm_xl.hip conv_xl), used where
# its 256-wide output tile is full: forward (with the BN moments) when
# Cout >= 256, stride-1 data gradient (a forward conv over flipped weights,
# optionally fused with the producer BN's backward reductions) when
# Cin >= 256.  ResNet-50 layers 3-4: forward 0.30-0.33 ms vs 0.46-0.49 (conv_nt)
# and dgrad 0.30-0.31 vs MIOpen 0.38-0.41 (profiles/conv3x3_xl_r2.md).
# DMP_DISABLE=xl_conv3 turns it off.
_XL3 = not _native.disabled("xl_conv3")
_STATS["xl_fwd"] = 0
_STATS["xl_dgrad"] = 0
_STATS["xl_bnbwd"] = 0


# Forward where none of our kernels wins (the layer-2 stride-2 3x3, other
# Cout < 256 shapes outside the halo kernels): the 4-wave conv_nt with fused
# moments (0.47-0.70 ms at batch 1024) loses to MIOpen's forward plus the
# separate BN moments pass (0.33-0.53 + 0.04-0.08 ms; profiles/conv3x3_xl_r2.md),
# so those run F.conv2d and let the BN reduce.  Tests set _MIOPEN_FWD = False
# to exercise conv_nt's forward.
_MIOPEN_FWD = True
_STATS["miopen_fwd"] = 0


# 3x3/s1/p1 convs with Cin = Cout = 64 on 56-wide maps (ResNet-50 layer 1)
# and 128 on 28-wide maps (layer 2) run on the persistent halo-tiled kernels
# (csrc/conv/conv3x3_halo.hip, conv3x3_c128.hip: weights in VGPRs, input halo
# in LDS, read once from HBM), forward with the BN moments fused and the data
# gradient as the same conv over flipped weights.  DMP_DISABLE=halo3 sends
# them back to the policy below.
_HALO3 = not _native.disabled("halo3")
_STATS["halo_fwd"] = 0
_STATS["halo_dgrad"] = 0


def _halo_kind(cin: int, cout: int, kh: int, kw: int, stride: int, pad: int, h: int, wdt: int) -> int:
    """64 / 128: which halo conv kernel runs this 3x3/s1/p1 conv; 0: none."""
    if not (_HALO3 and cin == cout and kh == 3 and kw == 3 and stride == 1 and pad == 1):
        return 0
    if cin == 64 and wdt == 56:
        return 64
    if cin == 128 and wdt == 28 and h % 4 == 0:
        return 128
    return 0


def _halo_conv(C, kind: int):
    return C.conv3x3_c64 if kind == 64 else C.conv3x3_c128


# The stride-2 block-0 3x3 of layer 2 (128 -> 128, 56 -> 28): data gradient as
# its four stride phases on the c128 halo kernel (conv3x3_c128.hip, PH).
_STATS["halo_dgrad_s2"] = 0


def _halo_dgrad_s2_ok(cin: int, cout: int, kh: int, kw: int, stride: int, pad: int, h: int, w: int) -> bool:
    return (_HALO3 and cin == 128 and cout == 128 and kh == 3 and kw == 3 and stride == 2 and pad == 1
            and w == 56 and h % 8 == 0)


# Weight gradients of every ResNet-50 3x3 (stride 1 and the stride-2 first
# blocks) on the persistent halo-tiled kernel: dW in registers, dy / x halo
# tiles streamed through LDS (csrc/conv/wgrad3x3.hip).  Stride 1 at batch 2048
# on MI355X (tools/wgrad_bench.py): 0.45-0.52 ms vs MIOpen's igemm_wrw 0.62-1.18 ms.
_STATS["halo_wgrad"] = 0


def _halo_wgrad_ok(C, cin: int, cout: int, kh: int, kw: int, stride: int, pad: int, h: int, w: int) -> bool:
    """h, w: INPUT size; the kernel covers stride 1 and 2 (even input sizes)."""
    return (kh == 3 and kw == 3 and stride in (1, 2) and pad == 1 and cin == cout and h == w
            and h % stride == 0 and C.wgrad3x3_supported(cin, h // stride, w // stride, stride))


def _miopen_fwd(cout: int, kh: int) -> bool:
    return _MIOPEN_FWD and kh > 1 and not _xl_fwd(cout, kh, kh)


# Cout = 128 (ResNet-50's layer-2 stride-2 3x3, the last MIOpen pass of the
# step) runs on the 4-wave kernel's 256 x 128 tile (four waves along M,
# gemm_xl_w4_kernel<EPI, 2, 4, 1>) with the BN moments fused.
_XL_N128 = True  # (tools/step_ab.py arms n128 / miopen)


def _xl_fwd(cout: int, kh: int, kw: int) -> bool:
    return _XL3 and (cout >= 256 or (cout == 128 and _XL_N128)) and kh == kw and kh > 1


def _xl_dgrad(cin: int, kh: int, kw: int, stride: int) -> bool:
    return _XL3 and cin >= 256 and stride == 1 and kh == kw and kh > 1


# Data gradient of the stride-2 3x3s of layers 3-4 (Cin = 256 / 512): four
# stride-phase implicit GEMMs on the ping-pong kernel writing straight into
# their pixels of dx (gemm_xl.hip conv_xl_dgrad_s2) -- no zero-filled dx and
# no zero taps, where MIOpen zero-fills dx and then runs its igemm_bwd.
_STATS["xl_dgrad_s2"] = 0
_PHASE_TAPS = ((1,), (2, 0))  # even / odd output phase: kernel taps, in offset order a = 0, 1


def _xl_dgrad_s2(cin: int, cout: int, kh: int, kw: int, stride: int, pad: int, h: int, w: int) -> bool:
    return (_XL3 and cin % 256 == 0 and cout % 64 == 0 and kh == 3 and kw == 3 and stride == 2 and pad == 1
            and h % 2 == 0 and w % 2 == 0)


def _phase_weights(weight: torch.Tensor):
    """[Cout, Cin, 3, 3] -> the four [Cin, taps * Cout] phase matrices (py, px)."""
    cin = weight.shape[1]
    w4 = weight.permute(1, 2, 3, 0)  # [Cin, 3, 3, Cout]
    out = []
    for py in (0, 1):
        for px in (0, 1):
            # stacked slices, not an index list: a list index is a host->device
            # copy, which a hipGraph capture (train/graphed.py) refuses
            taps = [w4[:, ky, kx] for ky in _PHASE_TAPS[py] for kx in _PHASE_TAPS[px]]
            out.append(torch.stack(taps, 1).reshape(cin, -1))
    return out


def _out_size(h: int, k: int, s: int, p: int) -> int:
    return (h + 2 * p - k) // s + 1


def _native_ok(x: torch.Tensor, w: torch.Tensor, groups: int, dilation) -> bool:
    if not ENABLED or not _native.gpu_path(x):
        return False
    return (groups == 1 and tuple(dilation) == (1, 1) and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 64 == 0
            and w.shape[0] % 64 == 0 and x.is_contiguous(memory_format=torch.channels_last))


def _wmat(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, kh, kw] -> [Cout, kh*kw*Cin] (a view for channels_last weights)."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1)


class _ConvIGFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, pad, moments, bn_slot=None):
        C = _native.require("conv_igemm")
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        ho, wo = _out_size(h, kh, stride, pad), _out_size(w, kw, stride, pad)
        mode = "moments" if moments else "store"
        y4 = None
        if moments is None:
            # MIOpen forward (layers whose native forward loses, finding 27); the
            # backward below still takes our kernels where they win (the halo
            # weight gradient of every stride-1 3x3)
            y4 = F.conv2d(x, weight, None, stride, pad)
            y2, mom = None, None
        elif _halo_kind(cin, cout, kh, kw, stride, pad, h, w):
            _STATS["halo_fwd"] += 1
            y2, mom = _halo_conv(C, _halo_kind(cin, cout, kh, kw, stride, pad, h, w))(
                x, _wmat(weight).contiguous(), moments)
            if not moments:
                mom = None
        elif _xl_fwd(cout, kh, kw):
            _STATS["xl_fwd"] += 1
            y2, mom = C.conv_xl(x, _wmat(weight), kh, kw, stride, pad, ho, wo, mode)
            if not moments:
                mom = None
        else:
            y2, mom = C.conv_nt(x, _wmat(weight), kh, kw, stride, pad, ho, wo, mode=mode)
        ctx.save_for_backward(x, weight)
        ctx.geo = (stride, pad, ho, wo)
        # x is a training-mode BN+ReLU output and our dgrad runs on conv_xl: its
        # epilogue can also do that BN's backward reductions (BnBwdSlot)
        ctx.bn_slot = bn_slot if (bn_slot is not None and _xl_dgrad(cin, kh, kw, stride)) else None
        if ctx.bn_slot is not None:
            bn_slot.consumers += 1
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        # the moments output never gets a gradient: do not let autograd build a
        # zero [2C+1] fp64 tensor for it every backward (one fill launch per layer)
        ctx.set_materialize_grads(False)
        if y4 is not None:
            return y4, mom
        return y2.view(n, ho, wo, cout).permute(0, 3, 1, 2), mom

    @staticmethod
    def backward(ctx, dy, _dmom):
        if dy is None:
            return (None,) * 6
        x, weight = ctx.saved_tensors
        C = _native.require("conv_igemm backward")
        stride, pad, ho, wo = ctx.geo
        n, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        bs, ctx.bn_slot = ctx.bn_slot, None
        hk = _halo_kind(cin, cout, kh, kw, stride, pad, h, w)
        if ctx.needs_input_grad[0] and hk:
            # dx = conv(dy, flip(W)^T): the same 3x3/s1/p1 C->C conv
            wfl = wt_cache.flipped(weight)
            _STATS["halo_dgrad"] += 1
            dx2, _ = _halo_conv(C, hk)(dy, wfl, False)
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        elif ctx.needs_input_grad[0] and _xl_dgrad(cin, kh, kw, stride):
            # dx = conv(dy, flip(W)^T, pad k-1-p) on the ping-pong implicit GEMM
            wfl = wt_cache.flipped(weight)
            _STATS["xl_dgrad"] += 1
            if bs is not None and bs.consumers == 1 and bs.x2 is not None:
                _STATS["xl_bnbwd"] += 1
                inv, bw, bb = (bs.invstd, bs.w32, bs.b32) if bs.y2 is None else (None, None, None)
                dx2, sums = C.conv_xl(dy, wfl, kh, kw, 1, kh - 1 - pad, h, w, "bnbwd", bn_x=bs.x2, bn_y=bs.y2,
                                      mean=bs.mean, invstd=inv, weight=bw, bias=bb)
                dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
                bs.park(dx, sums[: 2 * cin])
            else:
                dx2, _ = C.conv_xl(dy, wfl, kh, kw, 1, kh - 1 - pad, h, w, "store")
                dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        elif ctx.needs_input_grad[0] and _halo_dgrad_s2_ok(cin, cout, kh, kw, stride, pad, h, w):
            _STATS["halo_dgrad_s2"] += 1
            wt = weight.permute(1, 2, 3, 0).reshape(cin, -1).contiguous()
            dx = C.conv3x3_c128_dgrad_s2(dy, wt).view(n, h, w, cin).permute(0, 3, 1, 2)
        elif ctx.needs_input_grad[0] and _xl_dgrad_s2(cin, cout, kh, kw, stride, pad, h, w):
            _STATS["xl_dgrad_s2"] += 1
            dx2 = C.conv_xl_dgrad_s2(dy, _phase_weights(weight), h, w)
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        # weight gradients on the side stream (ops/wgrad_stream.py), beside the
        # data-gradient chain
        if ctx.needs_input_grad[1] and _halo_wgrad_ok(C, cin, cout, kh, kw, stride, pad, h, w):
            # persistent halo-tiled MFMA weight gradient (csrc/conv/wgrad3x3.hip)
            _STATS["halo_wgrad"] += 1
            with wgrad_stream.side(weight, dy, x):
                dw = C.wgrad3x3(dy, x, stride)
                if not weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous()
        if ctx.needs_input_grad[1] and dw is None and _xl_wgrad_ok(cin, kh, kw, n * ho * wo):
            _STATS["xl_wgrad"] += 1
            with wgrad_stream.side(weight, dy, x):
                dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
                g = C.conv_wgrad_xl(dy2, x, kh, kw, stride, pad, ho, wo, weight.dtype)
                dw = g.view(cout, kh, kw, cin).permute(0, 3, 1, 2)
                if not weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous()
        generic = NATIVE_BWD or _capturing()
        nat_d = ctx.needs_input_grad[0] and dx is None and generic
        nat_w = ctx.needs_input_grad[1] and dw is None and generic
        want_d = ctx.needs_input_grad[0] and not nat_d and dx is None
        want_w = ctx.needs_input_grad[1] and not nat_w and dw is None
        if want_d or want_w:
            # a weight-gradient-only library call also goes to the side stream
            with (wgrad_stream.side(weight, dy, x) if not want_d else contextlib.nullcontext()):
                dx_l, dw_l, _ = torch.ops.aten.convolution_backward(
                    dy, x, weight, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                    [want_d, want_w, False])
            if want_d:
                dx = dx_l
            if want_w:
                dw = dw_l
        if nat_d:
            wt = weight.permute(1, 2, 3, 0).reshape(cin, -1).contiguous()  # [Cin][kh][kw][Cout]
            dx2, _ = C.conv_nt(dy, wt, kh, kw, stride, pad, h, w, transposed=True)
            dx = dx2.view(n, h, w, cin).permute(0, 3, 1, 2)
        if nat_w:
            with wgrad_stream.side(weight, dy, x):
                dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
                g = C.conv_wgrad(dy2, x, kh, kw, stride, pad, ho, wo, weight.dtype)
                dw = g.view(cout, kh, kw, cin).permute(0, 3, 1, 2)
                if not weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous()
        return dx, dw, None, None, None, None


def conv2d_igemm(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, padding: int = 0,
                 moments: bool = False, groups: int = 1,
                 dilation=(1, 1)) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns (y, moments-or-None); moments = fp64 [2*Cout+1] of y (see BatchNormAct2d)."""
    if _native_ok(x, weight, groups, dilation) and _miopen_fwd(weight.shape[0], weight.shape[2]) and \
            not _capturing() and not \
            _halo_kind(x.shape[1], weight.shape[0], weight.shape[2], weight.shape[3], stride, padding, x.shape[2],
                       x.shape[3]):
        _STATS["miopen_fwd"] += 1
        geo = (x.shape[1], weight.shape[0], weight.shape[2], weight.shape[3], stride, padding, x.shape[2],
               x.shape[3])
        if torch.is_grad_enabled() and (weight.requires_grad or x.requires_grad) and (
                _halo_wgrad_ok(_native.native(), *geo) or _halo_dgrad_s2_ok(*geo) or _xl_dgrad_s2(*geo)):
            # MIOpen forward inside our Function so the backward can use the halo
            # weight gradient / the stride-phase data gradients
            y, _ = _ConvIGFn.apply(x, weight, stride, padding, None, None)
            return y, None
        return F.conv2d(x, weight, None, stride, padding, dilation, groups), None
    if _native_ok(x, weight, groups, dilation):
        _STATS["native"] += 1
        bn_slot = getattr(x, "_dmp_bnbwd", None) if torch.is_grad_enabled() else None
        y, mom = _ConvIGFn.apply(x, weight, stride, padding, moments, bn_slot)
        return y, (mom if moments else None)
    _STATS["torch"] += 1
    return F.conv2d(x, weight, None, stride, padding, dilation, groups), None


class ConvIG2d(nn.Conv2d):
    """Drop-in bias-free ``nn.Conv2d`` (square kernel, symmetric padding) routed
    through the implicit-GEMM MFMA kernels when the shape allows."""

    def __init__(self, cin: int, cout: int, kernel_size: int, stride: int = 1, padding: int = 0,
                 device=None, dtype=None):
        super().__init__(cin, cout, kernel_size, stride=stride, padding=padding, bias=False,
                         device=device, dtype=dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return conv2d_igemm(x, self.weight, self.stride[0], self.padding[0], False,
                            self.groups, self.dilation)[0]

    def forward_with_moments(self, x: torch.Tensor):
        return conv2d_igemm(x, self.weight, self.stride[0], self.padding[0], True,
                            self.groups, self.dilation)
