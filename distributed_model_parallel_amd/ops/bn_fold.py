"""BatchNorm folded through an expanding 1x1 convolution ("Gram fold").

The bottleneck's last stage is ``out = relu(bn3(a @ W^T) + residual)`` with
``a`` the 1x1 conv input [M, Cin] and ``W`` [Cout, Cin], Cout = 4 Cin.  Its
conv output y = a @ W^T is the widest tensor of the block, and the unfused
training step moves it through HBM five times (conv store, BN-apply read,
BN-backward read, BN-backward dx store, and the dx reads of the data / weight
gradient GEMMs).  Every quantity BN needs from y is, however, a small matrix
expression in W and two reductions of the 4x narrower ``a``:

  G = a^T a [Cin, Cin],   s = colsum(a) [Cin]
  forward    sum_m y[m, k]   = W[k] . s
             sum_m y[m, k]^2 = W[k] G W[k]^T            (BN mean / var)
             out = relu(acc * scale + shift + residual) in the GEMM epilogue
  backward   dz = dL/dout * [out > 0],  sdz = colsum dz,  D = dz^T a [Cout, Cin]
             sum_m dz[m, k] y[m, k] = D[k] . W[k]
             dy = al dz + be y + c  (per-channel al, be, c of the BN backward)
             dW = dy^T a = al o D + be o (W G) + c (x) s
             da = dy W   = [dz | a] @ [al o W ; W^T diag(be) W] + c^T W

so y is never written or read: the forward trades its store and re-read for
one Gram GEMM over ``a`` (G also serves the backward), and the backward's data
gradient becomes one GEMM over the concatenated operand [dz | a] (K grows by
Cin / Cout = 1/4) with the constant c^T W added in its epilogue -- where the
previous BN's backward reductions are fused as before (``BnBwdSlot``).  s
comes out of the previous BN's apply pass (``bn_forward_apply(...,
out_moments=True)``), D from the weight-gradient GEMM the conv ran anyway.

MI355X rationale: this moves the BN from HBM (the widest tensors of
ResNet-50 at ~5.5 TB/s) onto MFMA work sized Cin^2 per row -- exactly the
exchange CDNA4 rewards (2.5 PFLOP/s dense bf16 vs 8 TB/s).  Capability:
conv1x1 -> BatchNorm2d -> add -> ReLU of the reference's torchvision
Bottleneck (SURVEY.md north star N3); design: ours.

The statistics are exact algebra on the same bf16 operands the GEMM uses, so
they match the unfused BN up to fp32 accumulation order; the data gradient
rounds al o W and W^T diag(be) W to bf16 where the unfused path rounded dy.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import _native

_STATS = {"fold": 0, "fold_fused_bwd": 0, "fold_bnbwd_epilogue": 0}
ENABLED = not _native.disabled("bn_fold")


def stats() -> dict:
    return dict(_STATS)


def _rows(t: torch.Tensor) -> torch.Tensor:
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _unrows(t2: torch.Tensor, n: int, h: int, w: int) -> torch.Tensor:
    return t2.view(n, h, w, -1).permute(0, 3, 1, 2)


def _fold_stats(W: torch.Tensor, G: torch.Tensor, s: torch.Tensor, count: torch.Tensor):
    """Local BN moments [2Cout+1] (fp64) of y = a W^T, and W G (fp64)."""
    Wd = W.double()
    WG = Wd @ G.double()
    return torch.cat([Wd @ s, (WG * Wd).sum(1), count.reshape(1)]), WG


def _finalize(sums, w32, b32, rm, rv, momentum, eps, cout, nbt, native):
    if native:
        coef = _native.require("bn_fold").bn_finalize(sums, w32, b32, rm, rv, float(momentum), float(eps),
                                                       cout, nbt)
        return coef[0], coef[1], coef[2], coef[3]
    from .batchnorm import _finalize_torch
    if nbt is not None:
        nbt.add_(1)
    mean, invstd, scale, shift = _finalize_torch(sums, w32, b32, rm, rv, momentum, eps)
    return scale, shift, mean, invstd


def _xl_fwd(cout: int, cin: int) -> bool:
    from .conv1x1 import _xl
    return _xl(cout, cin)


class _ConvBNFoldFn(torch.autograd.Function):
    """out = relu(bn(conv1x1(a)) + residual), BN folded (module docstring)."""

    @staticmethod
    def forward(ctx, a, a_sums, weight, bn_w, bn_b, residual, running_mean, running_var, momentum, eps,
                nbt, reduce_moments, reduce_grads, relu, a_slot, out_slot):
        native = _native.gpu_path(a)
        n, cin, h, w = a.shape
        cout = weight.shape[0]
        a2 = _rows(a)
        W2 = weight.reshape(cout, cin)
        count = a_sums[2 * cin:2 * cin + 1]
        s = a_sums[:cin]
        if native:
            from .conv1x1 import _tn_xl
            C = _native.require("bn_fold")
            G = C.gemm_tn_xl(a2, a2, torch.float32) if _tn_xl(a2.shape[0], cin, cin) \
                else C.gemm_tn(a2, a2, torch.float32)
        else:
            ad = a2.double()
            G = ad.t() @ ad
        if native and C.bn_fold_supported(cout, cin):
            sums, WG = C.bn_fold_fwd(W2, G, a_sums)   # one launch: W G and the row dots
        else:
            sums, WG = _fold_stats(W2, G, s, count)
        if reduce_moments is not None:
            sums = reduce_moments(sums)
        w32 = bn_w.float() if bn_w is not None else None
        b32 = bn_b.float() if bn_b is not None else None
        rm = running_mean if (running_mean is not None and running_mean.dtype == torch.float32) else None
        rv = running_var if rm is not None else None
        scale, shift, mean, invstd = _finalize(sums, w32, b32, rm, rv, momentum, eps, cout, nbt, native)
        res2 = _rows(residual.to(a.dtype).contiguous(memory_format=torch.channels_last)) \
            if residual is not None else None
        if native:
            if _xl_fwd(cout, cin):
                out2, _ = C.gemm_xl_conv(a2, W2, "affine", residual=res2, scale=scale.contiguous(),
                                         shift=shift.contiguous(), relu=relu)
            else:
                out2, _ = C.gemm_nt(a2, W2, mode="affine", epi_scale=scale.contiguous(),
                                    epi_shift=shift.contiguous(), residual=res2, relu=relu)
        else:
            y = (a2.double() @ W2.double().t()).to(a.dtype).double()
            t = y * scale.double() + shift.double()
            if res2 is not None:
                t = t + res2.double()
            out2 = (t.clamp_min(0) if relu else t).to(a.dtype)
        ctx.save_for_backward(a, weight, out2, WG.float(), a_sums, mean, invstd, w32, sums[-1:])
        ctx.meta = (reduce_grads, relu, residual is not None, native, bn_w is not None, bn_b is not None,
                    bn_w.dtype if bn_w is not None else None)
        # a_slot: the producing BN's backward reductions can ride in our data-gradient epilogue
        ctx.a_slot = a_slot if native else None
        if ctx.a_slot is not None:
            a_slot.consumers += 1
        ctx.out_slot = None
        if out_slot is not None and native and relu:
            out_slot.y2 = out2     # mask source; x2 stays None: the consumer reduces sum dz only
            out_slot.mean = mean
            ctx.out_slot = out_slot
        ctx.set_materialize_grads(False)
        _STATS["fold"] += 1
        return _unrows(out2, n, h, w)

    @staticmethod
    def backward(ctx, dout):
        if dout is None:
            return (None,) * 16
        a, weight, out2, WG, asums, mean, invstd, w32, count = ctx.saved_tensors
        reduce_grads, relu, has_res, native, has_w, has_b, wdtype = ctx.meta
        n, cin, h, w = a.shape
        cout = weight.shape[0]
        a2 = _rows(a)
        W2 = weight.reshape(cout, cin)
        s = asums[:cin]
        slot = ctx.out_slot
        ctx.out_slot = None
        fused = slot.take(dout) if slot is not None else None
        dz2 = _rows(dout.contiguous(memory_format=torch.channels_last).to(a.dtype))
        if fused is not None:
            # the consumer's data-gradient epilogue applied the ReLU mask and reduced sum dz
            _STATS["fold_fused_bwd"] += 1
            sdz = fused[:cout]
        else:
            if relu:
                dz2 = torch.where(out2 > 0, dz2, torch.zeros((), dtype=dz2.dtype, device=dz2.device))
            sdz = dz2.sum(0, dtype=torch.float64)
        if native:
            from .conv1x1 import _tn_xl
            C = _native.require("bn_fold backward")
            D = C.gemm_tn_xl(dz2, a2, torch.float32) if _tn_xl(a2.shape[0], cout, cin) \
                else C.gemm_tn(dz2, a2, torch.float32)
        else:
            D = dz2.double().t() @ a2.double()
        if native and C.bn_fold_supported(cout, cin):
            # two launches: the row dots, then every coefficient-level output
            local = C.bn_fold_bwd_sums(D, W2, sdz.contiguous(), mean)
            sums = reduce_grads(local.clone()) if reduce_grads is not None else local
            dw2, dg, db, Bb, ebias = C.bn_fold_bwd_coef(sums, local, count, invstd, mean, w32, D,
                                                        WG, asums, W2)
            dw = dw2.view(cout, cin, 1, 1)
            if weight.is_contiguous(memory_format=torch.channels_last):
                dw = dw.contiguous(memory_format=torch.channels_last)
            da = _FoldDgrad.run(ctx, C, dz2, a2, Bb, ebias, n, cin, h, w) if ctx.needs_input_grad[0] else None
            gres = _unrows(dz2, n, h, w) if (has_res and ctx.needs_input_grad[5]) else None
            gw = dg.to(wdtype) if has_w and ctx.needs_input_grad[3] else None
            gb = db.to(wdtype) if has_b and ctx.needs_input_grad[4] else None
            return da, None, dw, gw, gb, gres, None, None, None, None, None, None, None, None, None, None
        Wd = W2.double()
        Dd = D.double()
        sdzx = (Dd * Wd).sum(1) - mean.double() * sdz
        local = torch.cat([sdz, sdzx])
        sums = local
        if reduce_grads is not None:
            sums = reduce_grads(local.clone())  # the reducer works in place
        cnt = count.reshape(()).double()
        istd = invstd.double()
        al = istd * (w32.double() if w32 is not None else 1.0)
        be = -al * istd * istd * sums[cout:] / cnt
        cc = -al * sums[:cout] / cnt - be * mean.double()
        dW = al[:, None] * Dd + be[:, None] * WG.double() + cc[:, None] * s[None, :]
        dw = dW.to(weight.dtype).view(cout, cin, 1, 1)
        if weight.is_contiguous(memory_format=torch.channels_last):
            dw = dw.contiguous(memory_format=torch.channels_last)
        # da = [dz | a] @ [al o W ; W^T diag(be) W] + c^T W
        Bm = torch.cat([(al[:, None] * Wd).t(), Wd.t() @ (be[:, None] * Wd)], 1)
        ebias = (cc @ Wd).float().contiguous()
        da = None
        if ctx.needs_input_grad[0]:
            if native:
                da = _FoldDgrad.run(ctx, C, dz2, a2, Bm.to(torch.bfloat16).contiguous(), ebias, n, cin, h, w)
            else:
                da2 = (torch.cat([dz2.double(), a2.double()], 1) @ Bm.t() + ebias.double()).to(a.dtype)
                da = _unrows(da2, n, h, w)
        gres = _unrows(dz2, n, h, w) if (has_res and ctx.needs_input_grad[5]) else None
        if reduce_grads is not None:
            dg, db = local[cout:] * istd, local[:cout]
        else:
            dg, db = sdzx * istd, sdz
        gw = dg.to(wdtype) if has_w and ctx.needs_input_grad[3] else None
        gb = db.to(wdtype) if has_b and ctx.needs_input_grad[4] else None
        return da, None, dw, gw, gb, gres, None, None, None, None, None, None, None, None, None, None


class _FoldDgrad:
    @staticmethod
    def run(ctx, C, dz2, a2, Bb, ebias, n, cin, h, w):
        """da = [dz | a] @ Bb^T + ebias on the MFMA GEMMs (two-source A operand);
        when ``a`` is a training-mode BN+ReLU output its backward reductions
        ride in the same epilogue (BnBwdSlot)."""
        cout = dz2.shape[1]
        bs = ctx.a_slot
        ctx.a_slot = None
        xl = _xl_fwd(cin, cout)
        if bs is not None and bs.consumers == 1 and bs.x2 is not None:
            _STATS["fold_bnbwd_epilogue"] += 1
            inv = bs.invstd if bs.y2 is None else None
            bw = bs.w32 if bs.y2 is None else None
            bb = bs.b32 if bs.y2 is None else None
            if xl:
                da2, asums = C.gemm_xl_conv(dz2, Bb, "bnbwd", bn_x=bs.x2, bn_y=bs.y2, mean=bs.mean,
                                            invstd=inv, weight=bw, bias=bb, a2=a2, ebias=ebias)
            else:
                da2, asums = C.gemm_nt_bnbwd(dz2, Bb, None, bs.x2, bs.y2, bs.mean, inv, bw, bb,
                                             a2=a2, ebias=ebias)
            da = _unrows(da2, n, h, w)
            bs.park(da, asums[: 2 * cin])
            return da
        if xl:
            da2, _ = C.gemm_xl_conv(dz2, Bb, "affine", a2=a2, shift=ebias)
        else:
            da2, _ = C.gemm_nt(dz2, Bb, mode="affine", epi_shift=ebias, a2=a2)
        return _unrows(da2, n, h, w)


def foldable(conv: nn.Module, bn: nn.Module, a: torch.Tensor) -> bool:
    """Training-mode conv1x1 -> BN(+residual)+ReLU that the fold covers natively."""
    from ..utils.checkpointing import in_recompute
    from .batchnorm import BatchNormAct2d
    from .conv1x1 import Conv1x1, _native_ok
    return (ENABLED and isinstance(bn, BatchNormAct2d) and bn.act == "relu" and bn.training
            and bn.track_running_stats and bn.momentum is not None and bn.running_mean is not None
            and bn.running_mean.dtype == torch.float32 and isinstance(conv, Conv1x1)
            and conv.stride[0] == 1 and torch.is_grad_enabled() and not in_recompute()
            and _native_ok(a, conv.weight) and conv.weight.shape[0] % 64 == 0 and a.shape[1] % 64 == 0)


def conv1x1_bn_fold(conv: nn.Module, bn: nn.Module, a: torch.Tensor, a_sums: torch.Tensor,
                    residual: Optional[torch.Tensor] = None, force: bool = False) -> torch.Tensor:
    """relu(bn(conv(a)) + residual) with the BN folded through the GEMM.

    ``a_sums``: fp64 [2Cin+1] (colsum a, colsum a^2, rows) -- from the producing
    BN apply (``BatchNormAct2d(..., out_moments=True)``).  ``force`` runs the
    fold on any device (the CPU path is the same algebra in fp64: tests)."""
    if not (force or foldable(conv, bn, a)):
        raise RuntimeError("conv1x1_bn_fold: configuration not covered (check foldable())")
    from .batchnorm import BnBwdSlot
    rmom, rgrad = bn._moment_reducers()
    a_slot = getattr(a, "_dmp_bnbwd", None)
    out_slot = BnBwdSlot() if _native.gpu_path(a) else None
    out = _ConvBNFoldFn.apply(a, a_sums, conv.weight, bn.weight, bn.bias, residual, bn.running_mean,
                              bn.running_var, bn.momentum, bn.eps, bn.num_batches_tracked, rmom, rgrad,
                              bn.act == "relu", a_slot, out_slot)
    if out_slot is not None and out_slot.ready():
        out._dmp_bnbwd = out_slot  # the next 1x1 conv's dgrad epilogue masks dz and reduces sum dz
    return out
