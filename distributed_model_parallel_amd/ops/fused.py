"""Cross-kernel fusions used by the models.

conv_bn: conv -> BatchNorm(+residual)(+ReLU) with the BN statistics produced by
the conv kernel's epilogue when both run natively (1x1 MFMA GEMM, implicit-GEMM
3x3 or depthwise 3x3); otherwise the plain two-module path.  In training this
removes the BN moments pass over the conv output (one full HBM read per layer).

GradSlot / grad_tap: a tensor x feeding two branches (a bottleneck's conv1 and
its shortcut) gets its gradient as the SUM of both branches' gradients --
autograd materialises both and launches an add kernel (3 full-tensor HBM
passes: the largest elementwise cost left in ResNet-50's backward).  Instead
the shortcut use goes through ``grad_tap(x, slot)``, whose backward parks its
gradient in the slot and returns None, and the consuming 1x1 conv adds the
parked gradient inside its data-gradient GEMM epilogue (C = acc + R).
A handshake keeps it correct under any backward order: the tap only parks
when a native consumer registered on the slot and has not run yet; otherwise
it returns the gradient and autograd sums as usual.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .batchnorm import BatchNormAct2d


class GradSlot:
    """Per-forward-call mailbox between a grad_tap and one native consumer.

    A stride-s 1x1 conv on the tapped branch (the ResNet downsample) may park
    its data gradient COMPACT -- [N*Ho*Wo, C] rows, the full-resolution
    gradient being zero off the stride grid -- with its geometry: no zero-filled
    full-size tensor, no scatter, and the consumer's epilogue reads 1/s^2 of the
    bytes (``res_map`` of gemm_nt_bnbwd / gemm_xl_conv)."""
    __slots__ = ("consumer", "consumer_ran", "grad", "compact", "compact_geom")

    def __init__(self):
        self.consumer = False      # a native conv registered to absorb the parked grad
        self.consumer_ran = False  # its backward already ran without a parked grad
        self.grad: Optional[torch.Tensor] = None
        self.compact: Optional[torch.Tensor] = None
        self.compact_geom = None

    def take(self) -> Optional[torch.Tensor]:
        g, self.grad = self.grad, None
        if g is None and self.compact is None:
            self.consumer_ran = True
        return g

    def take_compact(self):
        c, geom = self.compact, self.compact_geom
        self.compact = self.compact_geom = None
        return c, geom

    def can_park_compact(self) -> bool:
        return self.consumer and not self.consumer_ran and self.grad is None and self.compact is None


class _GradTap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        ctx.set_materialize_grads(False)  # a compact park leaves this output without a gradient
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        slot = ctx.slot
        if slot.consumer and not slot.consumer_ran and g is not None:
            slot.grad = g if slot.grad is None else slot.grad + g
            return None, None
        return g, None


def grad_tap(x: torch.Tensor, slot: Optional[GradSlot]) -> torch.Tensor:
    if slot is None or not slot.consumer or not (torch.is_grad_enabled() and x.requires_grad):
        return x
    out = _GradTap.apply(x, slot)
    out._dmp_gradslot = slot  # a strided 1x1 conv consuming `out` may park a compact gradient
    return out


def conv_bn(conv: nn.Module, bn: nn.Module, x: torch.Tensor,
            residual: Optional[torch.Tensor] = None,
            grad_slot: Optional[GradSlot] = None) -> torch.Tensor:
    fused = (isinstance(bn, BatchNormAct2d) and bn.training and hasattr(conv, "forward_with_moments"))
    if fused:
        if grad_slot is not None and getattr(conv, "accepts_grad_slot", False):
            y, sums = conv.forward_with_moments(x, grad_slot=grad_slot)
        else:
            y, sums = conv.forward_with_moments(x)
        return bn(y, residual, sums=sums)
    y = conv(x)
    if isinstance(bn, BatchNormAct2d):
        return bn(y, residual)
    if residual is not None:
        return bn(y) + residual
    return bn(y)


# --------------------------------------------------------------------------- #
# BN(+ReLU) applied inside the consuming 1x1 conv (training)
# --------------------------------------------------------------------------- #
class _BNReLUConv1x1Fn(torch.autograd.Function):
    """y = conv1x1(relu(bn(x))) with the BN output never materialised:

    forward   bn_finalize (coefficients from the fused moments, running stats),
              then the MFMA GEMM applies relu(x*scale + shift) while staging A
              (optionally emitting the moments of y for the next BN);
    backward  dgrad GEMM -> d(bn out); weight gradient GEMM re-applies the
              prologue while staging B; BN backward with the ReLU mask
              re-derived from x.  (Capability: conv(bn_relu(x)) as in the
              reference's torchvision ResNet-50; design: ours.)"""

    @staticmethod
    def forward(ctx, x, bn_w, bn_b, conv_w, sums, running_mean, running_var, momentum, eps, nbt,
                reduce_moments, reduce_grads, moments_out):
        from .. import _native
        from .conv1x1 import _rows, _unrows
        C = _native.require("bn_relu_conv1x1")
        n, cin, h, w = x.shape
        x2 = _rows(x)
        if reduce_moments is not None:
            sums = reduce_moments(sums)
        w32 = bn_w.float() if bn_w is not None else None
        b32 = bn_b.float() if bn_b is not None else None
        coef = C.bn_finalize(sums, w32, b32, running_mean, running_var, float(momentum), float(eps),
                             cin, nbt)
        scale, shift, mean, invstd = coef[0], coef[1], coef[2], coef[3]
        cout = conv_w.shape[0]
        y2, mom = C.gemm_nt(x2, conv_w.reshape(cout, cin), pro_scale=scale, pro_shift=shift,
                            mode="moments" if moments_out else "store")
        ctx.save_for_backward(x, conv_w, w32, b32, coef, sums[-1:])
        ctx.meta = (reduce_grads, bn_w.dtype if bn_w is not None else None, bn_w is not None,
                    bn_b is not None)
        if mom is None:
            mom = torch.empty(0, device=x.device, dtype=torch.float64)
        ctx.mark_non_differentiable(mom)
        ctx.set_materialize_grads(False)
        return _unrows(y2, n, h, w), mom

    @staticmethod
    def backward(ctx, dy, _dmom):
        if dy is None:
            return (None,) * 13
        from .. import _native
        from .conv1x1 import _rows, _unrows
        C = _native.require("bn_relu_conv1x1 backward")
        x, conv_w, w32, b32, coef, count = ctx.saved_tensors
        reduce_grads, wdtype, has_w, has_b = ctx.meta
        n, cin, h, w = x.shape
        cout = conv_w.shape[0]
        scale, shift, mean, invstd = coef[0], coef[1], coef[2], coef[3]
        x2 = _rows(x)
        dy2 = _rows(dy.contiguous(memory_format=torch.channels_last).to(x.dtype))
        w2 = conv_w.reshape(cout, cin)
        from .wt_cache import transposed
        g2, _ = C.gemm_nt(dy2, transposed(conv_w))            # d(relu(bn(x)))
        dw = C.gemm_tn(dy2, x2, conv_w.dtype, pro_scale=scale, pro_shift=shift).view(cout, cin, 1, 1)
        if conv_w.is_contiguous(memory_format=torch.channels_last):
            dw = dw.contiguous(memory_format=torch.channels_last)
        sums = C.bn_backward_moments(g2, x2, None, mean, True, cin, w32, b32, invstd)
        local = sums
        if reduce_grads is not None:
            local = sums.clone()  # the reducer works in place
            sums = reduce_grads(sums)
        dx2, dg, db, _ = C.bn_backward_apply(g2, x2, None, sums, count, w32, mean, invstd, True,
                                             True, False, cin, b32)
        if reduce_grads is not None:
            dg = (local[cin:] * invstd.double()).float()
            db = local[:cin].float()
        gw = dg.to(wdtype) if has_w and ctx.needs_input_grad[1] else None
        gb = db.to(wdtype) if has_b and ctx.needs_input_grad[2] else None
        return (_unrows(dx2, n, h, w), gw, gb, dw, None, None, None, None, None, None, None, None,
                None)


def bn_relu_conv1x1(bn: nn.Module, conv: nn.Module, x: torch.Tensor,
                    sums: Optional[torch.Tensor], moments_out: bool = True):
    """conv(relu(bn(x))) -> (y, moments-of-y or None).  Fused (BN apply + ReLU in
    the GEMM's operand staging) when training natively with fused input moments;
    otherwise the two modules run as usual."""
    from .. import _native
    from ..utils.checkpointing import in_checkpoint
    from .conv1x1 import Conv1x1, _native_ok
    if sums is None and isinstance(bn, BatchNormAct2d) and bn.training and _native_ok(x, conv.weight):
        # the producing conv ran on a library kernel (no fused moments): reduce here
        from .batchnorm import _as_rows, local_moments
        sums = local_moments(_as_rows(x)[0], True)
    fusable = (sums is not None and isinstance(bn, BatchNormAct2d) and bn.act == "relu"
               and bn.training and bn.track_running_stats and bn.momentum is not None
               and not in_checkpoint() and isinstance(conv, Conv1x1) and conv.stride[0] == 1
               and bn.running_mean is not None and bn.running_mean.dtype == torch.float32
               and _native_ok(x, conv.weight) and torch.is_grad_enabled())
    if not fusable:
        y = bn(x, sums=sums)
        return conv.forward_with_moments(y) if moments_out else (conv(y), None)
    rmom, rgrad = bn._moment_reducers()
    nbt = bn.num_batches_tracked
    y, mom = _BNReLUConv1x1Fn.apply(x, bn.weight, bn.bias, conv.weight, sums, bn.running_mean,
                                    bn.running_var, bn.momentum, bn.eps, nbt, rmom, rgrad,
                                    moments_out)
    _STATS_FUSED["bn_relu_conv1x1"] += 1
    return y, (mom if moments_out else None)


_STATS_FUSED = {"bn_relu_conv1x1": 0}


# --------------------------------------------------------------------------- #
# Stem: BN(+ReLU) applied inside the 3x3/s2 max pool (training)
# --------------------------------------------------------------------------- #
class _BNReLUMaxPoolFn(torch.autograd.Function):
    """pool(relu(bn(x))) with the BN output never materialised:

    forward   bn_finalize (coefficients + running stats from the conv's fused
              moments), then the pool normalises each tap on load
              (``maxpool2d_bn_forward``);
    backward  the pool's gather backward also masks with the ReLU (from x)
              and reduces the BN backward's (sum dz, sum dz*(x-mean))
              (``maxpool2d_bn_backward``); the BN apply pass then reads dz, x.
    Saves the BN apply pass forward (write + re-read of the stem activation,
    the largest tensor of the network) and the moments pass backward."""

    @staticmethod
    def forward(ctx, x, bn_w, bn_b, sums, running_mean, running_var, momentum, eps, nbt, reduce_moments,
                reduce_grads, k, s, p):
        from .. import _native
        C = _native.require("bn_relu_maxpool")
        c = x.shape[1]
        if reduce_moments is not None:
            sums = reduce_moments(sums)
        w32 = bn_w.float() if bn_w is not None else None
        b32 = bn_b.float() if bn_b is not None else None
        coef = C.bn_finalize(sums, w32, b32, running_mean, running_var, float(momentum), float(eps), c, nbt)
        y, idx = C.maxpool2d_bn_forward(x, coef[0].contiguous(), coef[1].contiguous(), k, s, p)
        ctx.save_for_backward(x, idx, w32, b32, coef, sums[-1:])
        ctx.meta = (reduce_grads, bn_w.dtype if bn_w is not None else None, bn_w is not None,
                    bn_b is not None, k, s, p)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .. import _native
        from .batchnorm import backward_apply
        C = _native.require("bn_relu_maxpool backward")
        x, idx, w32, b32, coef, count = ctx.saved_tensors
        reduce_grads, wdtype, has_w, has_b, k, s, p = ctx.meta
        c = x.shape[1]
        scale, shift, mean, invstd = (coef[i].contiguous() for i in range(4))
        dz, sums = C.maxpool2d_bn_backward(dy.contiguous(memory_format=torch.channels_last), idx, x,
                                           scale, shift, mean, k, s, p)
        sums = sums[: 2 * c]
        local = sums
        if reduce_grads is not None:
            local = sums.clone()  # the reducer works in place
            sums = reduce_grads(sums)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, c)
        dz2 = dz.permute(0, 2, 3, 1).reshape(-1, c)
        dx2, dg, db, _ = backward_apply(dz2, x2, None, sums, count, w32, mean, invstd, True, False, False,
                                        True, b32)
        if reduce_grads is not None:
            dg = (local[c:] * invstd.double()).float()
            db = local[:c].float()
        n, _, h, w = x.shape
        gx = dx2.view(n, h, w, c).permute(0, 3, 1, 2)
        gw = dg.to(wdtype) if has_w and ctx.needs_input_grad[1] else None
        gb = db.to(wdtype) if has_b and ctx.needs_input_grad[2] else None
        return gx, gw, gb, None, None, None, None, None, None, None, None, None, None, None


_STATS_FUSED["bn_relu_maxpool"] = 0


class _StemBNReLUMaxPoolFn(torch.autograd.Function):
    """pool(relu(bn(stem_conv(img)))) with the stem's BN backward apply folded
    into its weight gradient (the image needs no gradient).

    The BN backward's output dx = a*dz + b*y + c (per-channel a, b, c from the
    reduced sums; y the conv output, dz the pool-scattered, ReLU-masked
    gradient) feeds ONLY the stem's weight gradient dW = dx^T P (P the
    implicit patch matrix of the space-to-depth image).  That is linear in dx:

        dW[o, k] = a_o (dz^T P)[o, k] + b_o (y^T P)[o, k] + c_o colsum(P)[k]

    so the step runs the halo weight-gradient kernel on dz and on y (fp32
    outputs) plus a column sum of P (one pass over the small s2d image)
    instead of writing dx -- the 2048 x 64 x 112 x 112 apply pass (1.85 ms at
    batch 2048, its read of dz and y and its write of dx) is gone.  b*(y^T P)
    and c*colsum(P) partly cancel (through the mean); both are fp32 sums."""

    @staticmethod
    def forward(ctx, img, wmat, bn_w, bn_b, running_mean, running_var, momentum, eps, nbt, reduce_moments,
                reduce_grads, pad):
        from .. import _native
        from .stem import _STATS as _STEM_STATS
        C = _native.require("stem + bn + maxpool")
        _STEM_STATS["native"] += 1  # the same halo stem kernels as StemConv2d's own path
        _STEM_STATS["halo"] += 1
        n, _, h, w = img.shape
        ho, wo = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
        s = C.space_to_depth2(img, 3)
        y2, sums = C.stem_halo_fwd(s, wmat.contiguous(), ho, True)
        co = wmat.shape[0]
        y = y2.view(n, ho, wo, co).permute(0, 3, 1, 2)
        if reduce_moments is not None:
            sums = reduce_moments(sums)
        w32 = bn_w.float() if bn_w is not None else None
        b32 = bn_b.float() if bn_b is not None else None
        coef = C.bn_finalize(sums, w32, b32, running_mean, running_var, float(momentum), float(eps), co, nbt)
        out, idx = C.maxpool2d_bn_forward(y, coef[0].contiguous(), coef[1].contiguous(), 3, 2, pad)
        ctx.save_for_backward(s, y, idx, w32, b32, coef, sums[-1:])
        ctx.meta = (reduce_grads, bn_w.dtype if bn_w is not None else None, bn_w is not None, bn_b is not None,
                    pad, n, ho, wo, wmat.dtype)
        ctx.mark_non_differentiable(idx)
        return out

    @staticmethod
    def backward(ctx, dy):
        from .. import _native
        C = _native.require("stem + bn + maxpool backward")
        s, y, idx, w32, b32, coef, count = ctx.saved_tensors
        reduce_grads, wdtype, has_w, has_b, pad, n, ho, wo, mdtype = ctx.meta
        co = y.shape[1]
        scale, shift, mean, invstd = (coef[i].contiguous() for i in range(4))
        dz, sums = C.maxpool2d_bn_backward(dy.contiguous(memory_format=torch.channels_last), idx, y,
                                           scale, shift, mean, 3, 2, pad)
        sums = sums[: 2 * co]
        local = sums
        if reduce_grads is not None:
            local = sums.clone()  # the reducer works in place
            sums = reduce_grads(sums)
        sdz, sdzx = sums[:co], sums[co:]
        istd = invstd.double()
        rows = lambda t: t.permute(0, 2, 3, 1).reshape(n * ho * wo, co)  # noqa: E731
        t_dz = C.stem_halo_wgrad(rows(dz), s, ho, torch.float32)
        t_y = C.stem_halo_wgrad(rows(y), s, ho, torch.float32)
        # colsum(P)[r*64 + q*16 + ch] = sum over images and output pixels of s[n, ch, oh+r, ow+q]:
        # the batch sum of the (channels-last) s2d image as one column reduction; its 4 x 4
        # window sums (fp64), the BN-backward coefficients al / be / cc and
        # dW = al t_dz + be t_y + cc colsum(P) in one launch (stem_halo.hip stem_fold_finish)
        hs, ws = s.shape[2], s.shape[3]
        img = s.permute(0, 2, 3, 1).reshape(n, -1).sum(0, dtype=torch.float32).view(hs, ws, -1)
        dw = C.stem_fold_finish(img.contiguous(), ho, wo, t_dz, t_y, sums.contiguous(),
                                count.reshape(1).to(torch.float64), invstd.float().contiguous(),
                                None if w32 is None else w32.float().contiguous(), mean.float().contiguous(), mdtype)
        if reduce_grads is not None:
            dg = (local[co:] * invstd.double()).float()
            db = local[:co].float()
        else:
            dg, db = (sdzx * istd).float(), sdz.float()
        gw = dg.to(wdtype) if has_w and ctx.needs_input_grad[2] else None
        gb = db.to(wdtype) if has_b and ctx.needs_input_grad[3] else None
        return None, dw, gw, gb, None, None, None, None, None, None, None, None


_STATS_FUSED["stem_bn_relu_maxpool"] = 0


def _stem_fold_ok(conv: nn.Module, x: torch.Tensor) -> bool:
    from .. import _native
    from .stem import StemConv2d, _HALO, _native_ok
    if not (_FUSE_STEM_WGRAD and _HALO and isinstance(conv, StemConv2d) and _native_ok(conv, x)):
        return False
    C = _native.native()
    n, _, h, w = x.shape
    ho, wo = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
    return C.stem_halo_supported((h + 7) // 2, (w + 7) // 2, ho, wo) and conv.out_channels == 64


def conv_bn_maxpool(conv: nn.Module, bn: nn.Module, pool: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """pool(bn_relu(conv(x))) -- the ResNet stem.  BN apply + ReLU run inside the
    pool (forward) and the BN backward's reductions inside the pool's backward
    when training natively; otherwise the modules run one after another."""
    from .. import _native
    from ..utils.checkpointing import in_checkpoint
    fusable = (isinstance(bn, BatchNormAct2d) and bn.act == "relu" and bn.training and bn.track_running_stats
               and bn.momentum is not None and not in_checkpoint() and torch.is_grad_enabled()
               and hasattr(conv, "forward_with_moments") and isinstance(pool, nn.MaxPool2d)
               and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2))
               and pool.padding in (0, 1, (1, 1), (0, 0)) and not pool.ceil_mode
               and pool.dilation in (1, (1, 1)) and _FUSE_STEM_POOL)
    if not fusable:
        return pool(conv_bn(conv, bn, x))
    pad = pool.padding if isinstance(pool.padding, int) else pool.padding[0]
    if _stem_fold_ok(conv, x) and bn.running_mean is not None and bn.running_mean.dtype == torch.float32:
        from .stem import stem_wmat
        rmom, rgrad = bn._moment_reducers()
        _STATS_FUSED["stem_bn_relu_maxpool"] += 1
        _STATS_FUSED["bn_relu_maxpool"] += 1
        return _StemBNReLUMaxPoolFn.apply(x, stem_wmat(conv.weight), bn.weight, bn.bias, bn.running_mean,
                                          bn.running_var, bn.momentum, bn.eps, bn.num_batches_tracked, rmom,
                                          rgrad, pad)
    y, sums = conv.forward_with_moments(x)
    if (sums is None or not _native.gpu_path(y) or y.dtype != torch.bfloat16
            or not y.is_contiguous(memory_format=torch.channels_last)
            or y.shape[1] < 8 or y.shape[1] % 8 != 0 or 128 % (y.shape[1] // 8) != 0
            or bn.running_mean is None or bn.running_mean.dtype != torch.float32):
        return pool(bn(y, sums=sums))
    rmom, rgrad = bn._moment_reducers()
    _STATS_FUSED["bn_relu_maxpool"] += 1
    return _BNReLUMaxPoolFn.apply(y, bn.weight, bn.bias, sums, bn.running_mean, bn.running_var, bn.momentum,
                                  bn.eps, bn.num_batches_tracked, rmom, rgrad, 3, 2, pad)


from .. import _native as _nat  # noqa: E402
_FUSE_STEM_POOL = not _nat.disabled("fuse_stem_pool")
# DMP_DISABLE=fuse_stem_wgrad: keep the stem's BN backward apply pass (A/B runs)
_FUSE_STEM_WGRAD = not _nat.disabled("fuse_stem_wgrad")
