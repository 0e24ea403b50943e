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
from . import wt_cache

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


# finalize fused into the folded-moments kernel (bn_fold_fwd_finalize) when no
# SyncBN reduce sits between them (tools/step_ab.py arms finf / finsep)
_FUSED_FINALIZE = True


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


def _xl_dgrad(cin: int, cout: int) -> bool:
    """Folded data gradient [M, cout + cin] @ Bb^T -> [M, cin]: the ping-pong
    GEMM (x2 kernel at cin = 128) from cin >= 128 -- measured 1.09 / 1.19 /
    1.24x the NT kernel at layers 2 / 3 / 4 (batch 2048; 1.02 / 1.30 / 0.96 at
    256), 0.53x at layer 1's cin = 64 (profiles/raw_r4/fold_dgrad_ab_r4aa.md)."""
    from .conv1x1 import _XL
    return _XL and cin >= 128 and cin % 128 == 0 and cout >= 512


def _map_rows(x2: torch.Tensor, geom, n: int):
    """The rows of x2 [N*Hi*Wi, C] a stride-s 1x1 conv reads (CPU path)."""
    if not geom:
        return x2
    s, ho, wo, hi, wi = geom
    return x2.view(n, hi, wi, -1)[:, ::s, ::s].reshape(n * ho * wo, -1)


class _FoldMeta:
    """Non-tensor configuration of one folded call: per BN (running_mean,
    running_var, momentum, eps, num_batches_tracked, reduce_moments,
    reduce_grads), the downsample stride, the BnBwdSlots and the GradSlot
    that may take the shortcut's gradient compact."""
    __slots__ = ("bn", "relu", "stride", "a_slot", "out_slot", "x_park")

    def __init__(self, bn, relu, stride=1, a_slot=None, out_slot=None, x_park=None):
        self.bn, self.relu, self.stride = bn, relu, stride
        self.a_slot, self.out_slot, self.x_park = a_slot, out_slot, x_park


def _bn_spec(bn: nn.Module):
    rmom, rgrad = bn._moment_reducers()
    return (bn.running_mean, bn.running_var, bn.momentum, bn.eps, bn.num_batches_tracked, rmom, rgrad)


class _ConvBNFoldFn(torch.autograd.Function):
    """out = relu(bn3(conv3(a)) + residual)              (one branch), or
    out = relu(bn3(conv3(a)) + bn_d(conv_d(x_s)))        (two: the downsample
    folded too -- one GEMM over [a | x_s], x_s = x sampled at the stride),
    BNs folded (module docstring)."""

    @staticmethod
    def forward(ctx, meta, a, a_sums, w3, g3, b3, x, wd, gd, bd, residual):
        native = _native.gpu_path(a)
        C = _native.require("bn_fold") if native else None
        n, cin, h, w = a.shape
        cout = w3.shape[0]
        a2 = _rows(a)
        br = [dict(inp=a2, asums=a_sums, W=w3.reshape(cout, cin), Wp=w3, g=g3, b=b3, spec=meta.bn[0], geom=[])]
        if x is not None:
            cx, hi, wi = x.shape[1], x.shape[2], x.shape[3]
            from .conv1x1 import _geom
            geom = _geom(meta.stride, hi, wi)
            x2 = _rows(x)
            xs = C.bn_fold_colsum(x2, geom) if native else _cpu_moments(_map_rows(x2, geom, n))
            br.append(dict(inp=x2, asums=xs, W=wd.reshape(cout, cx), Wp=wd, g=gd, b=bd, spec=meta.bn[1],
                           geom=geom))
        for b in br:
            b.update(_fold_branch_forward(C, b, n, native))
        if native:
            xl = _xl_fwd(cout, cin)
            if len(br) == 1:
                res2 = _rows(residual.to(a.dtype).contiguous(memory_format=torch.channels_last)) \
                    if residual is not None else None
                if xl:
                    out2, _ = C.gemm_xl_conv(a2, br[0]["W"], "affine", residual=res2, scale=br[0]["scale"],
                                             shift=br[0]["shift"], relu=meta.relu)
                else:
                    out2, _ = C.gemm_nt(a2, br[0]["W"], mode="affine", epi_scale=br[0]["scale"],
                                        epi_shift=br[0]["shift"], residual=res2, relu=meta.relu)
            else:
                # both BN scales folded into the operand, the shifts summed: one GEMM over [a | x_s]
                Bf, shift = C.bn_fold_scale_concat(br[0]["W"], br[0]["scale"], br[0]["shift"], br[1]["W"],
                                                   br[1]["scale"], br[1]["shift"])
                if xl:
                    out2, _ = C.gemm_xl_conv(a2, Bf, "affine", shift=shift, relu=meta.relu, a2=br[1]["inp"],
                                             a2_map=br[1]["geom"])
                else:
                    out2, _ = C.gemm_nt(a2, Bf, mode="affine", epi_shift=shift, relu=meta.relu, a2=br[1]["inp"],
                                        a2_map=br[1]["geom"])
        else:
            t = 0.0
            for b in br:
                y = (_map_rows(b["inp"], b["geom"], n).double() @ b["W"].double().t()).to(a.dtype).double()
                t = t + y * b["scale"].double() + b["shift"].double()
            if residual is not None:
                t = t + _rows(residual).double()
            out2 = (t.clamp_min(0) if meta.relu else t).to(a.dtype)
        saved = [a, x, w3, wd, out2]
        for b in br:
            saved += [b["WG"], b["asums"], b["mean"], b["invstd"], b["w32"], b["count"]]
        ctx.save_for_backward(*saved)
        ctx.nbr = len(br)
        ctx.geoms = [b["geom"] for b in br]
        ctx.meta = meta
        ctx.native = native
        ctx.has_res = residual is not None
        ctx.wdtypes = (g3.dtype if g3 is not None else None, gd.dtype if gd is not None else None)
        if native and meta.a_slot is not None:
            meta.a_slot.consumers += 1  # the producing BN's reductions can ride in our dgrad epilogue
        if native and meta.out_slot is not None and meta.relu:
            meta.out_slot.y2 = out2     # mask source; x2 stays None: the consumer reduces sum dz only
            meta.out_slot.mean = br[0]["mean"]
        else:
            meta.out_slot = None
        ctx.set_materialize_grads(False)
        _STATS["fold" if len(br) == 1 else "fold_ds"] += 1
        return _unrows(out2, n, h, w)

    @staticmethod
    def backward(ctx, dout):
        nret = 11
        if dout is None:
            return (None,) * nret
        a, x, w3, wd, out2 = ctx.saved_tensors[:5]
        rest = ctx.saved_tensors[5:]
        meta, native = ctx.meta, ctx.native
        C = _native.require("bn_fold backward") if native else None
        n, cin, h, w = a.shape
        cout = w3.shape[0]
        a2 = _rows(a)
        slot = meta.out_slot
        meta.out_slot = None
        fused = slot.take(dout) if slot is not None else None
        dz2 = _rows(dout.contiguous(memory_format=torch.channels_last).to(a.dtype))
        if fused is not None:
            # the consumer's data-gradient epilogue applied the ReLU mask and reduced sum dz
            _STATS["fold_fused_bwd"] += 1
            sdz = fused[:cout]
        elif native and dz2.shape[1] <= 2048:
            # one pass: mask, store dz and reduce sum dz (the network's last block,
            # whose gradient comes from the pooling: 1.3 ms of torch where / cast /
            # fp64 sum at batch 2048 before, profiles/README.md finding 41)
            if meta.relu:
                dz2, s = C.bn_fold_relu_mask(dz2.contiguous(), out2.contiguous())
            else:
                s = C.bn_fold_colsum(dz2.contiguous())
            sdz = s[:cout]
        else:
            if meta.relu:
                dz2 = torch.where(out2 > 0, dz2, torch.zeros((), dtype=dz2.dtype, device=dz2.device))
            sdz = dz2.sum(0, dtype=torch.float64)
        inputs = [(a2, w3.reshape(cout, cin))]
        if x is not None:
            inputs.append((_rows(x), wd.reshape(cout, x.shape[1])))
        grads = []
        for i, (inp, W) in enumerate(inputs):
            WG, asums, mean, invstd, w32, count = rest[6 * i:6 * i + 6]
            grads.append(_fold_branch_backward(C, dz2, sdz, inp, ctx.geoms[i], n, W, WG, asums, mean, invstd, w32,
                                               count, meta.bn[i][6], native))
        wdt3, wdtd = ctx.wdtypes
        # a: the data gradient of conv3 ([dz | a] @ Bm^T + c^T W), with the producing BN's reductions
        da = None
        if ctx.needs_input_grad[1]:
            Bm, eb = grads[0]["Bm"], grads[0]["ebias"]
            if native:
                da = _FoldDgrad.run(meta, C, dz2, a2, Bm, eb, n, cin, h, w)
            else:
                da2 = (torch.cat([dz2.double(), a2.double()], 1) @ Bm.double().t() + eb.double()).to(a.dtype)
                da = _unrows(da2, n, h, w)
        dw3 = _wgrad_view(grads[0]["dW"], w3)
        gg3 = grads[0]["dg"].to(wdt3) if wdt3 is not None and ctx.needs_input_grad[4] else None
        gb3 = grads[0]["db"].to(wdt3) if wdt3 is not None and ctx.needs_input_grad[5] else None
        dx = dwd = ggd = gbd = None
        if x is not None:
            gd_ = grads[1]
            dwd = _wgrad_view(gd_["dW"], wd)
            ggd = gd_["dg"].to(wdtd) if wdtd is not None and ctx.needs_input_grad[8] else None
            gbd = gd_["db"].to(wdtd) if wdtd is not None and ctx.needs_input_grad[9] else None
            if ctx.needs_input_grad[6]:
                dx = _fold_shortcut_dgrad(meta, C, dz2, _rows(x), x.shape, gd_, ctx.geoms[1], native, n)
        gres = _unrows(dz2, n, h, w) if (ctx.has_res and ctx.needs_input_grad[10]) else None
        return None, da, None, dw3, gg3, gb3, dx, dwd, ggd, gbd, gres


def _cpu_moments(x2: torch.Tensor) -> torch.Tensor:
    xd = x2.double()
    return torch.cat([xd.sum(0), (xd * xd).sum(0), xd.new_tensor([float(x2.shape[0])])])


def _gram(C, inp, geom, native, n):
    if not native:
        xd = _map_rows(inp, geom, n).double()
        return xd.t() @ xd
    from .conv1x1 import _tn_xl, _tn_xl_strided
    if geom:
        s, ho, wo, hi, wi = geom
        c = inp.shape[1]
        if _tn_xl_strided(n * ho * wo, c, c) and C.gram_strided_xl_supported(n, c, hi, wi, ho, wo):
            # both operands the sampled rows, gathered in place by the 4-wave TN kernel
            _STATS["fold_ds_gram_xl"] = _STATS.get("fold_ds_gram_xl", 0) + 1
            return C.gram_strided_xl(inp.view(n, hi, wi, c).permute(0, 3, 1, 2), s, ho, wo)
        return C.gemm_tn(inp, inp, torch.float32, b_map=geom, a_mapped=True)
    c = inp.shape[1]
    return C.gemm_tn_xl(inp, inp, torch.float32) if _tn_xl(inp.shape[0], c, c) else C.gemm_tn(inp, inp, torch.float32)


def _fold_branch_forward(C, b, n, native):
    """Gram, folded moments, (cross-rank reduce), finalize of one branch."""
    W, asums, geom = b["W"], b["asums"], b["geom"]
    cout, cin = W.shape
    rm, rv, momentum, eps, nbt, rmom, _ = b["spec"]
    G = _gram(C, b["inp"], geom, native, n)
    w32 = b["g"].float() if b["g"] is not None else None
    b32 = b["b"].float() if b["b"] is not None else None
    rm = rm if (rm is not None and rm.dtype == torch.float32) else None
    rv = rv if rm is not None else None
    Wf = wt_cache.as_f32(b["Wp"]) if (native and "Wp" in b) else None
    if native and C.bn_fold_supported(cout, cin) and rmom is None and _FUSED_FINALIZE and C.get_fold_gemm() in (1, 2):
        # W G, the row dots and the BN finalize in one launch (no cross-rank moment reduce in between)
        sums, WG, coef = C.bn_fold_fwd_finalize(W, G, asums, Wf, w32, b32, rm, rv, float(momentum), float(eps), nbt)
        scale, shift, mean, invstd = coef[0], coef[1], coef[2], coef[3]
    else:
        if native and C.bn_fold_supported(cout, cin):
            # W G and the row dots (the fp32 W from the optimizer-driven cache when it holds one)
            sums, WG = C.bn_fold_fwd(W, G, asums, Wf)
        else:
            sums, WG = _fold_stats(W, G, asums[:cin], asums[2 * cin:2 * cin + 1])
        if rmom is not None:
            sums = rmom(sums)
        scale, shift, mean, invstd = _finalize(sums, w32, b32, rm, rv, momentum, eps, cout, nbt, native)
    return dict(WG=WG.float(), scale=scale.contiguous(), shift=shift.contiguous(), mean=mean, invstd=invstd,
                w32=w32, count=sums[-1:])


def _fold_branch_backward(C, dz2, sdz, inp, geom, n, W, WG, asums, mean, invstd, w32, count, reduce_grads, native):
    """dW, dgamma, dbeta, the dgrad operand Bm = [(al o W)^T | W^T diag(be) W] and c^T W of one branch."""
    cout, cin = W.shape
    if native:
        from .conv1x1 import _tn_xl, _tn_xl_strided
        if geom and _tn_xl_strided(dz2.shape[0], cout, cin):
            # the strided branch's sampled rows read in place by the 4-wave
            # TN kernel's tap gather (a 1x1 / stride-s "conv" weight gradient)
            s, ho, wo, hi, wi = geom
            x4 = inp.view(n, hi, wi, cin).permute(0, 3, 1, 2)
            D = C.conv_wgrad_xl(dz2, x4, 1, 1, s, 0, ho, wo, torch.float32)
            _STATS["fold_ds_wgrad_xl"] = _STATS.get("fold_ds_wgrad_xl", 0) + 1
        elif geom:
            D = C.gemm_tn(dz2, inp, torch.float32, b_map=geom)
        else:
            D = C.gemm_tn_xl(dz2, inp, torch.float32) if _tn_xl(inp.shape[0], cout, cin) \
                else C.gemm_tn(dz2, inp, torch.float32)
    else:
        D = dz2.double().t() @ _map_rows(inp, geom, n).double()
    if native and C.bn_fold_supported(cout, cin):
        # two launches: the row dots, then every coefficient-level output
        local = C.bn_fold_bwd_sums(D, W, sdz.contiguous(), mean)
        sums = reduce_grads(local.clone()) if reduce_grads is not None else local
        dW, dg, db, Bm, eb = C.bn_fold_bwd_coef(sums, local, count, invstd, mean, w32, D, WG, asums, W)
        return dict(dW=dW, dg=dg, db=db, Bm=Bm, ebias=eb)
    Wd = W.double()
    Dd = D.double()
    sdzx = (Dd * Wd).sum(1) - mean.double() * sdz
    local = torch.cat([sdz, sdzx])
    sums = reduce_grads(local.clone()) if reduce_grads is not None else local  # the reducer works in place
    cnt = count.reshape(()).double()
    istd = invstd.double()
    al = istd * (w32.double() if w32 is not None else 1.0)
    be = -al * istd * istd * sums[cout:] / cnt
    cc = -al * sums[:cout] / cnt - be * mean.double()
    dW = al[:, None] * Dd + be[:, None] * WG.double() + cc[:, None] * asums[:cin][None, :]
    Bm = torch.cat([(al[:, None] * Wd).t(), Wd.t() @ (be[:, None] * Wd)], 1)
    if native:
        Bm = Bm.to(torch.bfloat16).contiguous()
    return dict(dW=dW.to(W.dtype), dg=(local[cout:] * istd).float(), db=local[:cout].float(), Bm=Bm,
                ebias=(cc @ Wd).float().contiguous())


def _wgrad_view(dW, weight):
    dw = dW.to(weight.dtype).view(weight.shape)
    if weight.is_contiguous(memory_format=torch.channels_last):
        dw = dw.contiguous(memory_format=torch.channels_last)
    return dw


def _fold_shortcut_dgrad(meta, C, dz2, x2, xshape, g, geom, native, n):
    """Gradient of the folded downsample branch w.r.t. the block input x:
    dx_s = [dz | x_s] @ Bm_d^T + c_d^T W_d on the stride grid.  A strided
    branch parks it COMPACT in the GradSlot of conv1's data gradient (which
    adds it in its epilogue, ops/fused.py); stride 1 returns it through
    autograd (the grad_tap parks it)."""
    nx, cx, hi, wi = xshape
    cout = dz2.shape[1]
    if native:
        if _xl_fwd(cx, cout):
            dxs, _ = C.gemm_xl_conv(dz2, g["Bm"], "affine", a2=x2, a2_map=geom, shift=g["ebias"])
        else:
            dxs, _ = C.gemm_nt(dz2, g["Bm"], mode="affine", epi_shift=g["ebias"], a2=x2, a2_map=geom)
    else:
        xs = _map_rows(x2, geom, n).double()
        dxs = (torch.cat([dz2.double(), xs], 1) @ g["Bm"].double().t() + g["ebias"].double()).to(x2.dtype)
    if not geom:
        return _unrows(dxs, nx, hi, wi)
    ps = meta.x_park
    meta.x_park = None
    if ps is not None and ps.can_park_compact():
        _STATS["fold_ds_compact"] += 1
        ps.compact, ps.compact_geom = dxs, list(geom)
        return None
    s, ho, wo = geom[0], geom[1], geom[2]
    full = torch.zeros(nx * hi * wi, cx, device=dxs.device, dtype=dxs.dtype)
    full.view(nx, hi, wi, cx)[:, ::s, ::s].copy_(dxs.view(nx, ho, wo, cx))
    return _unrows(full, nx, hi, wi)


class _FoldDgrad:
    @staticmethod
    def run(meta, C, dz2, a2, Bb, ebias, n, cin, h, w):
        """da = [dz | a] @ Bb^T + ebias on the MFMA GEMMs (two-source A operand);
        when ``a`` is a training-mode BN+ReLU output its backward reductions
        ride in the same epilogue (BnBwdSlot)."""
        cout = dz2.shape[1]
        bs = meta.a_slot
        meta.a_slot = None
        xl = _xl_dgrad(cin, cout)
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
    from ..utils.checkpointing import in_checkpoint
    from .batchnorm import BatchNormAct2d
    from .conv1x1 import Conv1x1, _native_ok
    return (ENABLED and isinstance(bn, BatchNormAct2d) and bn.act == "relu" and bn.training
            and bn.track_running_stats and bn.momentum is not None and bn.running_mean is not None
            and bn.running_mean.dtype == torch.float32 and isinstance(conv, Conv1x1)
            and conv.stride[0] == 1 and torch.is_grad_enabled() and not in_checkpoint()
            and _native_ok(a, conv.weight) and conv.weight.shape[0] % 64 == 0 and a.shape[1] % 64 == 0)


def conv1x1_bn_fold(conv: nn.Module, bn: nn.Module, a: torch.Tensor, a_sums: torch.Tensor,
                    residual: Optional[torch.Tensor] = None, force: bool = False,
                    downsample: Optional[nn.Module] = None, x: Optional[torch.Tensor] = None) -> torch.Tensor:
    """relu(bn(conv(a)) + residual) with the BN folded through the GEMM, or --
    with ``downsample`` (Sequential(Conv1x1(stride s), BatchNormAct2d)) and the
    block input ``x`` instead of ``residual`` -- relu(bn(conv(a)) +
    bn_d(conv_d(x))) with both BNs folded into one GEMM over [a | x_s].

    ``a_sums``: fp64 [2Cin+1] (colsum a, colsum a^2, rows) -- from the producing
    BN apply (``BatchNormAct2d(..., out_moments=True)``).  ``force`` runs the
    fold on any device (the CPU path is the same algebra in fp64: tests)."""
    if not (force or foldable(conv, bn, a)):
        raise RuntimeError("conv1x1_bn_fold: configuration not covered (check foldable())")
    from .batchnorm import BnBwdSlot
    native = _native.gpu_path(a)
    two = downsample is not None
    if two and residual is not None:
        raise ValueError("conv1x1_bn_fold: residual and downsample are exclusive")
    specs = [_bn_spec(bn)]
    cd = bd = None
    if two:
        cd, bd = downsample[0], downsample[1]
        specs.append(_bn_spec(bd))
    meta = _FoldMeta(specs, bn.act == "relu", stride=cd.stride[0] if two else 1,
                     a_slot=getattr(a, "_dmp_bnbwd", None) if native else None,
                     out_slot=BnBwdSlot() if native else None,
                     x_park=getattr(x, "_dmp_gradslot", None) if two else None)
    out = _ConvBNFoldFn.apply(meta, a, a_sums, conv.weight, bn.weight, bn.bias, x if two else None,
                              cd.weight if two else None, bd.weight if two else None, bd.bias if two else None,
                              residual)
    if meta.out_slot is not None and meta.out_slot.ready():
        out._dmp_bnbwd = meta.out_slot  # the next 1x1 conv's dgrad epilogue masks dz and reduces sum dz
    return out


def foldable_downsample(ds: Optional[nn.Module], x: torch.Tensor, cout: int) -> bool:
    """A ResNet downsample (Sequential(Conv1x1, BatchNormAct2d without ReLU))
    that can join the bn3 fold: the same checks as foldable() on its BN, the
    block input as its conv's native operand, Cin <= 1024 for the coefficient kernels."""
    from ..utils.checkpointing import in_checkpoint
    from .batchnorm import BatchNormAct2d
    from .conv1x1 import Conv1x1, _native_ok
    if not (ENABLED and _FOLD_DS and isinstance(ds, nn.Sequential) and len(ds) == 2):
        return False
    conv, bn = ds[0], ds[1]
    return (isinstance(conv, Conv1x1) and isinstance(bn, BatchNormAct2d) and bn.act is None and bn.training
            and bn.track_running_stats and bn.momentum is not None and bn.running_mean is not None
            and bn.running_mean.dtype == torch.float32 and torch.is_grad_enabled() and not in_checkpoint()
            and _native_ok(x, conv.weight) and conv.weight.shape[0] == cout and x.shape[1] % 64 == 0
            and x.shape[1] <= 1024)


_FOLD_DS = not _native.disabled("bn_fold_ds")
_STATS.update({"fold_ds": 0, "fold_ds_compact": 0})
