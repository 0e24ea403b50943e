"""1x1 convolution on channels-last activations as an MFMA GEMM
(``csrc/conv/gemm_bf16.hip``), optionally emitting the BatchNorm moments of its
output so the following BN skips its statistics pass.

  forward   y[M, Cout] = x[M, Cin] @ W[Cout, Cin]^T        (our MFMA kernel,
            optional fused per-channel (sum, sum^2) of y)
  dgrad     dx[M, Cin] = dy[M, Cout] @ W                    (our MFMA kernel)
  wgrad     dW[Cout, Cin] = dy^T @ x                        (our split-M MFMA
            kernel with ds_read_b64_tr_b16 transposes; fp32 partials)

Stride-2 1x1 convs (ResNet downsample) address the sampled rows in place
through a row map (forward / wgrad read them, dgrad scatters into them): no
subsample copy, no scatter pass.  Anything the kernel does not cover (CPU, fp32, channel counts not multiple of 8) uses
``F.conv2d``.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


from .. import _native
from . import grad_accum, wgrad_stream, wt_cache

_STATS = {"native": 0, "torch": 0, "fused_dgrad": 0, "fused_bn_bwd": 0, "xl": 0, "compact_dgrad": 0,
          "compact_residual": 0}


def _native_ok(x: torch.Tensor, w: torch.Tensor) -> bool:
    if not _native.gpu_path(x):
        return False
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.dim() == 4
            and x.shape[1] % 8 == 0 and w.shape[0] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


def _rows(x: torch.Tensor) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _unrows(y2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return y2.view(n, h, w, -1).permute(0, 3, 1, 2)


def _blaslt_dgrad(m: int, cin: int, cout: int) -> bool:
    """Plain data gradients (no fused epilogue) where hipBLASLt measured faster than
    our NT kernel on MI355X (tools/microbench.py --wgrad, profiles/conv1x1_backends.md):
    reduction depth (cout) >= 1024 over <= 64K rows -- ResNet-50 layer3/4 conv3."""
    return cout >= 1024 and m <= 65536


# A/B switches (measured per box): compact strided shortcut gradients, glds-ring GEMMs
_COMPACT = not _native.disabled("compact_shortcut")
_XL = not _native.disabled("xl_conv")


def _xl(n: int, k: int) -> bool:
    """Output width N, reduction K of a 1x1-conv GEMM where the ping-pong
    kernel (gemm_xl_conv) measured faster than the 4-wave NT kernel with the
    same epilogue: N >= 256 with K >= 128.  Round 2 kept N = 256 / K > 512 on
    NT (profiles/conv1x1_xl.md); after the round-4 epilogue changes layer 3's
    conv1 forward (N = 256, K = 1024) runs 1.24x faster on it at batch 2048 and
    1.31x at 256 (profiles/raw_r4/fold_dgrad_ab_r4ac.md).  Narrow N (<= 128)
    and K = 64 stay on NT."""
    return _XL and k >= 128 and k % 64 == 0 and n >= 256
# (N = 128 stays on gemm_nt's 128 x 128 tile: on the 4-wave 256 x 128 tile
# the forward with moments measured no faster, 114.18 vs 114.08 ms at batch
# 2048, and the x2 kernel slower, 113.45 vs 113.28: finding 75)


def _geom(stride: int, hi: int, wi: int):
    """Row map [s, Ho, Wo, Hi, Wi] the kernels use to address a stride-s grid in place."""
    if stride == 1:
        return []
    return [stride, (hi - 1) // stride + 1, (wi - 1) // stride + 1, hi, wi]


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, stride, moments, slot, bn_slot=None, park_slot=None):
        C = _native.require("conv1x1")
        n, cin, h, w = x.shape
        geom = _geom(stride, h, w)
        ho, wo = (geom[1], geom[2]) if geom else (h, w)
        w2 = weight.reshape(weight.shape[0], cin)
        # strided convs read the sampled rows in place (no subsample copy)
        if moments and not geom and _xl(w2.shape[0], cin):
            _STATS["xl"] += 1
            y2, mom = C.gemm_xl_conv(_rows(x), w2, "moments")
        else:
            y2, mom = C.gemm_nt(_rows(x), w2, mode="moments" if moments else "store", a_map=geom)
        ctx.save_for_backward(x, weight)
        ctx.geom = geom
        ctx.slot = slot
        # x is a training-mode BN+ReLU output: our dgrad epilogue can also do
        # that BN's backward reductions (ops/batchnorm.py BnBwdSlot)
        ctx.bn_slot = bn_slot if (bn_slot is not None and not geom) else None
        # strided conv on a grad_tap'ed branch: may park its dgrad compact (ops/fused.py)
        ctx.park_slot = park_slot if geom else None
        if ctx.bn_slot is not None:
            bn_slot.consumers += 1
        if slot is not None and not geom:
            slot.consumer = True  # our dgrad epilogue will absorb the shortcut's gradient
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        # the moments output never gets a gradient: do not let autograd build a
        # zero [2C+1] fp64 tensor for it every backward (one fill launch per layer)
        ctx.set_materialize_grads(False)
        return _unrows(y2, n, ho, wo), mom

    @staticmethod
    def backward(ctx, dy, _dmom):
        if dy is None:
            return (None,) * 7
        x, weight = ctx.saved_tensors
        C = _native.require("conv1x1 backward")
        n, cin, h, w = x.shape
        cout = weight.shape[0]
        dy2 = _rows(dy.contiguous(memory_format=torch.channels_last).to(x.dtype))
        w2 = weight.reshape(cout, cin)
        dx = dw = None
        ps = ctx.park_slot
        ctx.park_slot = None
        if ctx.needs_input_grad[0] and ps is not None and ps.can_park_compact():
            # the consumer adds the stride-grid rows itself: no zero-filled full-size dx
            _STATS["compact_dgrad"] += 1
            ps.compact, _ = C.gemm_nt(dy2, wt_cache.transposed(weight))
            ps.compact_geom = list(ctx.geom)
        elif ctx.needs_input_grad[0]:
            # strided: the GEMM scatters into the sampled rows of a zeroed full-size grad
            extra = ctx.slot.take() if (ctx.slot is not None and ctx.slot.consumer) else None
            cextra, cgeom = ctx.slot.take_compact() if ctx.slot is not None else (None, None)
            bs = ctx.bn_slot
            ctx.bn_slot = None
            if cextra is not None and not (bs is not None and bs.consumers == 1 and bs.ready()):
                # no fused BN epilogue to read it compact: expand to full resolution
                full = torch.zeros(n * h * w, cin, device=dy.device, dtype=x.dtype)
                full.view(n, h, w, cin)[:, ::cgeom[0], ::cgeom[0]].copy_(cextra.view(n, cgeom[1], cgeom[2], cin))
                extra = full.view(n, h, w, cin).permute(0, 3, 1, 2) if extra is None else extra + full.view(
                    n, h, w, cin).permute(0, 3, 1, 2)
                cextra = None
            if bs is not None and bs.consumers == 1 and bs.ready():
                # dz = relu_mask * (dy @ W (+ shortcut grad)) and the producer BN's
                # (sum dz, sum dz*(x-mean)) in ONE epilogue pass
                _STATS["fused_bn_bwd"] += 1
                if extra is not None:
                    _STATS["fused_dgrad"] += 1
                    extra = _rows(extra.to(x.dtype).contiguous(memory_format=torch.channels_last))
                # mask affine (x*invstd*w + b - mean*invstd*w > 0) is formed in the epilogue
                inv = bs.invstd if bs.y2 is None else None
                bw = bs.w32 if bs.y2 is None else None
                bb = bs.b32 if bs.y2 is None else None
                rmap = []
                if cextra is not None:
                    if extra is not None:  # both a full and a compact parked gradient: expand
                        full = torch.zeros(n * h * w, cin, device=dy.device, dtype=x.dtype)
                        full.view(n, h, w, cin)[:, ::cgeom[0], ::cgeom[0]].copy_(
                            cextra.view(n, cgeom[1], cgeom[2], cin))
                        extra = extra + full
                    else:
                        extra, rmap = cextra, [cgeom[0], cgeom[1], cgeom[2], h, w]
                        _STATS["compact_residual"] += 1
                if _xl(cin, cout):
                    _STATS["xl"] += 1
                    dx2, sums = C.gemm_xl_conv(dy2, wt_cache.transposed(weight), "bnbwd", residual=extra,
                                               bn_x=bs.x2, bn_y=bs.y2, mean=bs.mean, invstd=inv,
                                               weight=bw, bias=bb, res_map=rmap)
                else:
                    dx2, sums = C.gemm_nt_bnbwd(dy2, wt_cache.transposed(weight), extra, bs.x2, bs.y2,
                                                bs.mean, inv, bw, bb, rmap)
                dx = _unrows(dx2, n, h, w)
                bs.park(dx, sums[: 2 * cin])
                dx2 = None
            elif extra is not None:  # dx = dy @ W + (the shortcut branch's gradient), one pass
                _STATS["fused_dgrad"] += 1
                extra = _rows(extra.to(x.dtype).contiguous(memory_format=torch.channels_last))
                dx2, _ = C.gemm_nt(dy2, wt_cache.transposed(weight), mode="add", residual=extra)
            elif not ctx.geom and _blaslt_dgrad(dy2.shape[0], cin, cout):
                dx2 = dy2 @ w2  # deep-K / short-M: hipBLASLt's stream-K tiles win here
            else:
                dx2, _ = C.gemm_nt(dy2, wt_cache.transposed(weight), c_map=ctx.geom)
            if dx2 is not None:
                dx = _unrows(dx2, n, h, w)
        if ctx.needs_input_grad[1]:
            # split-M MFMA GEMM with transposing LDS reads (hipBLASLt picks a 4-tile,
            # no-split kernel for this tiny-output / huge-reduction shape); the
            # ping-pong form where both output dims fill its 256x256 tile.  On the
            # weight-gradient side stream, beside the data-gradient chain.
            # inside grad_accum.accumulate_param_grads the split-K reduce adds
            # straight into weight.grad (micro-batch accumulation, no autograd add)
            acc = grad_accum.target(weight)
            with wgrad_stream.side(weight, dy2, x):
                if not ctx.geom and _tn_xl(dy2.shape[0], cout, cin):
                    _STATS["tn_xl"] += 1
                    dw = C.gemm_tn_xl(dy2, _rows(x), weight.dtype, out=acc).view(cout, cin, 1, 1)
                elif ctx.geom and _tn_xl_strided(dy2.shape[0], cout, cin):
                    # stride-s 1x1 (ResNet downsample): the 4-wave TN kernel's
                    # tap gather reads the sampled rows of x in place
                    _STATS["tn_xl_strided"] += 1
                    s, ho, wo = ctx.geom[0], ctx.geom[1], ctx.geom[2]
                    dw = C.conv_wgrad_xl(dy2, x, 1, 1, s, 0, ho, wo, weight.dtype, out=acc).view(cout, cin, 1, 1)
                else:
                    dw = C.gemm_tn(dy2, _rows(x), weight.dtype, b_map=ctx.geom, out=acc).view(cout, cin, 1, 1)
                if acc is not None:
                    dw = None
                elif weight.is_contiguous(memory_format=torch.channels_last):
                    dw = dw.contiguous(memory_format=torch.channels_last)
        return dx, dw, None, None, None, None, None


_TN_XL = not _native.disabled("tn_xl")
_STATS["tn_xl"] = 0


# (16k -> 8k rows with the narrow tiles: ResNet-50 layer 4 at batch 256,
# 12544 rows, joins the 4-wave kernel; tools/step_ab.py tnmin8k 19.95 vs
# tnmin16k 20.02 ms, tnmin4k 19.94)
_TN_XL_MIN_ROWS = 8_192
_TN_XL_MIN_CH = 64  # narrower sides take the 64-wide narrow tile (tools/step_ab.py arms tnch16 / tnch64)


def _tn_xl(m: int, cout: int, cin: int) -> bool:
    """1x1 weight gradients on gemm_tn_xl, whose default main loop is the
    4-wave kernel (gemm_tn_w4, finding 70): at batch 2048 it beats the split-M
    gemm_tn on every ResNet-50 shape, 1.15x on the 64-wide layer-1 ones
    (0.78 vs 0.89 ms) to 1.9x on layer 4 (0.19 vs 0.36 ms), and hipBLASLt by
    2-5x (tools/pipe_bench.py --only wgrad).  Until round 5 (8-wave ping-pong
    loop) only >= 256-wide shapes from 100k rows took it.  (The 224-px
    convergence test lowers the row threshold so its batch-64 run trains this
    route.)"""
    return _TN_XL and cout >= _TN_XL_MIN_CH and cin >= _TN_XL_MIN_CH and m >= _TN_XL_MIN_ROWS


_STATS["tn_xl_strided"] = 0


def _tn_xl_strided(m: int, cout: int, cin: int) -> bool:
    """Strided 1x1 weight gradients on the tap-gather TN kernel (conv_wgrad_xl,
    Cin % 256 == 0): the ResNet-50 downsample convs, which the split-M TN
    kernel took through its row map."""
    return _TN_XL and cout >= 64 and cin % 256 == 0 and m >= _TN_XL_MIN_ROWS


def conv1x1(x: torch.Tensor, weight: torch.Tensor, stride: int = 1,
            moments: bool = False, grad_slot=None) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Returns (y, moments-or-None); moments = fp64 [2*Cout+1] of y (see BatchNormAct2d).
    grad_slot (ops.fused.GradSlot): absorb a shortcut branch's gradient of x
    into this conv's data-gradient epilogue."""
    if _native_ok(x, weight):
        _STATS["native"] += 1
        bn_slot = getattr(x, "_dmp_bnbwd", None) if torch.is_grad_enabled() else None
        park = getattr(x, "_dmp_gradslot", None) if (_COMPACT and torch.is_grad_enabled() and stride != 1) \
            else None
        y, mom = _Conv1x1Fn.apply(x, weight, stride, moments, grad_slot, bn_slot, park)
        return y, (mom if moments else None)
    _STATS["torch"] += 1
    return F.conv2d(x, weight, None, stride), None


class Conv1x1(nn.Conv2d):
    """Drop-in ``nn.Conv2d(cin, cout, 1, stride, bias=False)``."""
    accepts_grad_slot = True

    def __init__(self, cin: int, cout: int, stride: int = 1, device=None, dtype=None):
        super().__init__(cin, cout, 1, stride=stride, bias=False, device=device, dtype=dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return conv1x1(x, self.weight, self.stride[0])[0]

    def forward_with_moments(self, x: torch.Tensor, grad_slot=None):
        return conv1x1(x, self.weight, self.stride[0], moments=True, grad_slot=grad_slot)
