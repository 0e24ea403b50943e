"""Fused BatchNorm(+residual)(+ReLU) for channels-last activations.

``BatchNormAct2d`` is a drop-in ``nn.BatchNorm2d`` (same parameters, buffers
and state_dict keys) whose forward can also add a residual and apply ReLU in
the same pass.  On MI355X it runs the HIP kernels of ``csrc/bn/batchnorm.hip``
on the [N*H*W, C] view of a channels-last tensor (2 HBM passes forward, 2
backward, ReLU re-derived from the saved output).  On CPU the same two-phase
algorithm runs in PyTorch ops, which is also what makes the SyncBatchNorm
variant testable over gloo.

The two-phase structure (local moments -> optional all-reduce -> finalize ->
apply) is shared with :class:`..parallel.sync_batchnorm.SyncBatchNorm`,
which plugs a cross-rank reduction between the phases (SURVEY.md D11;
reference Readme.md:151).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from . import grad_accum
from ..utils.checkpointing import in_recompute

# A moment reducer maps local fp64 moments [2C+1] = (sum x, sum x^2, rows) to
# the global ones (an all-reduce SUM); identity for plain BN.  The row count
# travels inside the tensor, so nothing ever syncs the host.
MomentReducer = Callable[[torch.Tensor], torch.Tensor]
GradReducer = Callable[[torch.Tensor], torch.Tensor]

_STATS = {"native_fwd": 0, "torch_fwd": 0}
_INF = float("inf")
# activation -> upper clip of the (clipped) ReLU the BN kernels apply
ACTS = {None: None, "relu": _INF, "relu6": 6.0}

# BN backward reductions fused into the consuming 1x1 conv's data-gradient
# epilogue (BnBwdSlot); DMP_DISABLE=fuse_bn_bwd turns it off for A/B runs.
_FUSE_BWD = not _native.disabled("fuse_bn_bwd")


def stats() -> dict:
    return dict(_STATS)


# --------------------------------------------------------------------------- #
# Layout helpers
# --------------------------------------------------------------------------- #
def _as_rows(x: torch.Tensor) -> Tuple[torch.Tensor, Callable[[torch.Tensor], torch.Tensor]]:
    """View/convert x to a row-major [M, C] matrix and return an inverse map."""
    if x.dim() == 2:
        x2 = x.contiguous()
        return x2, lambda t: t
    if x.dim() == 4:
        n, c, h, w = x.shape
        xl = x.contiguous(memory_format=torch.channels_last)
        x2 = xl.permute(0, 2, 3, 1).reshape(-1, c)
        return x2, lambda t: t.view(n, h, w, c).permute(0, 3, 1, 2)
    if x.dim() == 3:  # [N, C, L] (BatchNorm1d on sequences)
        n, c, l = x.shape
        x2 = x.transpose(1, 2).contiguous().reshape(-1, c)
        return x2, lambda t: t.view(n, l, c).transpose(1, 2)
    raise ValueError(f"BatchNorm expects 2-D, 3-D or 4-D input, got {x.dim()}-D")


def _native_ok(x2: torch.Tensor) -> bool:
    if not _native.gpu_path(x2):
        return False
    c = x2.shape[1]
    vec = 8 if x2.dtype == torch.bfloat16 else 4
    return (x2.dtype in (torch.float32, torch.bfloat16) and c % vec == 0
            and x2.data_ptr() % 16 == 0 and x2.is_contiguous())


# --------------------------------------------------------------------------- #
# Primitive ops: native (HIP) or PyTorch reference, identical math
# --------------------------------------------------------------------------- #
def local_moments(x2: torch.Tensor, native: bool) -> torch.Tensor:
    c = x2.shape[1]
    if native:
        return _native.require("bn").bn_local_moments(x2, c)
    xd = x2.double()
    return torch.cat([xd.sum(0), (xd * xd).sum(0), xd.new_tensor([float(x2.shape[0])])])


def forward_apply(x2, sums, weight, bias, rm, rv, momentum, eps, res2, relu, native, nbt=None,
                  out_moments=False, clip=_INF):
    """Training-mode normalise from (global) moments; updates running stats and
    increments `nbt` (num_batches_tracked) -- inside the kernel when native.

    Returns (y, mean, invstd) [+ fp64 (colsum y, colsum y^2, rows) with out_moments]."""
    c = x2.shape[1]
    if native:
        return _native.require("bn").bn_forward_apply(x2, sums, weight, bias, rm, rv,
                                                       float(momentum), float(eps), res2, relu, c,
                                                       nbt, out_moments, clip)
    if nbt is not None:
        nbt.add_(1)
    mean, invstd, scale, shift = _finalize_torch(sums, weight, bias, rm, rv, momentum, eps)
    y = _apply_torch(x2, scale, shift, res2, relu, clip)
    if out_moments:
        yd = y.double()
        return [y, mean, invstd, torch.cat([yd.sum(0), (yd * yd).sum(0), yd.new_tensor([float(y.shape[0])])])]
    return [y, mean, invstd]


def eval_apply(x2, rm, rv, weight, bias, eps, res2, relu, native, clip=_INF):
    c = x2.shape[1]
    if native:
        return _native.require("bn").bn_eval_apply(x2, rm, rv, weight, bias, float(eps), res2,
                                                    relu, c, clip)
    invstd = torch.rsqrt(rv.float() + eps)
    w = weight.float() if weight is not None else torch.ones_like(invstd)
    b = bias.float() if bias is not None else torch.zeros_like(invstd)
    scale = w * invstd
    shift = b - rm.float() * scale
    return [_apply_torch(x2, scale, shift, res2, relu, clip), rm.float(), invstd]


def _finalize_torch(sums, weight, bias, rm, rv, momentum, eps):
    c = (sums.numel() - 1) // 2
    count = sums[2 * c]
    mean = sums[:c] / count
    var = (sums[c:2 * c] / count - mean * mean).clamp_min(0)
    invstd = torch.rsqrt(var + eps).float()
    w = weight.float() if weight is not None else torch.ones_like(invstd)
    b = bias.float() if bias is not None else torch.zeros_like(invstd)
    scale = w * invstd
    shift = b - mean.float() * scale
    if rm is not None:
        unbiased = var * count / (count - 1.0).clamp_min(1.0)
        rm.mul_(1 - momentum).add_(mean.to(rm.dtype), alpha=momentum)
        rv.mul_(1 - momentum).add_(unbiased.to(rv.dtype), alpha=momentum)
    return [mean.float(), invstd, scale, shift]


def _apply_torch(x2, scale, shift, res2, relu, clip=_INF):
    y = x2.float() * scale + shift
    if res2 is not None:
        y = y + res2.float()
    if relu:
        y = y.clamp(0, clip)
    return y.to(x2.dtype)


def _relu_mask(x2, y2, mean, invstd, weight, bias, clip=_INF):
    """(Clipped) ReLU mask of the forward output: 0 < y < clip, or -- when y was
    not saved (no residual fused) -- re-derived from x with the forward's
    per-channel affine."""
    if y2 is not None:
        return (y2 > 0) & (y2 < clip)
    sc = invstd * (weight if weight is not None else 1.0)
    sh = (bias if bias is not None else 0.0) - mean * sc
    t = torch.addcmul(sh, x2.float(), sc)
    return (t > 0) & (t < clip)


def backward_moments(dy2, x2, y2, mean, relu, native, weight=None, bias=None, invstd=None, clip=_INF):
    c = x2.shape[1]
    if native:
        return _native.require("bn").bn_backward_moments(dy2, x2, y2, mean, relu, c, weight, bias,
                                                          invstd, clip)
    dz = dy2.double()
    if relu:
        dz = dz * _relu_mask(x2, y2, mean, invstd, weight, bias, clip)
    return torch.cat([dz.sum(0), (dz * (x2.double() - mean.double())).sum(0)])


def backward_apply(dy2, x2, y2, sums, count, weight, mean, invstd, training, relu, want_dres, native,
                   bias=None, clip=_INF, acc_weight=None, acc_bias=None):
    """`count` is a 1-element fp64 tensor (global rows).  y2 None with relu:
    mask from x (see _relu_mask).  acc_weight / acc_bias (native only): fp32
    gradients the affine gradients are added into (then returned as None)."""
    c = x2.shape[1]
    if native:
        return _native.require("bn").bn_backward_apply(dy2, x2, y2, sums, count, weight, mean,
                                                        invstd, training, relu, want_dres, c, bias,
                                                        clip, acc_weight, acc_bias)
    count = count.reshape(()).to(torch.float64)
    sdz, sdzx = sums[:c], sums[c:]
    w = weight.double() if weight is not None else torch.ones_like(sdz)
    istd = invstd.double()
    dz = dy2.double()
    if relu:
        dz = dz * _relu_mask(x2, y2, mean, invstd, weight, bias, clip)
    a = w * istd
    if training:
        b = -a * istd * istd * sdzx / count
        cc = -a * sdz / count - b * mean.double()
        dx = a * dz + b * x2.double() + cc
    else:
        dx = a * dz
    dres = dz.to(x2.dtype) if want_dres else None
    return [dx.to(x2.dtype), (sdzx * istd).float(), sdz.float(), dres]


# --------------------------------------------------------------------------- #
# Backward fusion handshake with the consuming 1x1 conv
# --------------------------------------------------------------------------- #
class BnBwdSlot:
    """Mailbox between a training-mode BN+ReLU and the ONE native 1x1 conv that
    consumes its output (attached to the output tensor as ``_dmp_bnbwd``).

    The conv's data-gradient GEMM produces this BN's incoming gradient G; with
    the slot it also applies the ReLU mask and reduces (sum dz, sum dz*(x-mean))
    in its epilogue (``gemm_nt_bnbwd``) and parks the result here.  The BN
    backward uses the parked sums -- skipping its own moments pass over dy and
    x -- only if the gradient it receives IS the conv's output, unmodified
    (same storage, same version): any other contribution summed in by autograd
    makes it fall back to the full computation (still correct, since the mask
    is idempotent)."""
    __slots__ = ("x2", "y2", "mean", "invstd", "w32", "b32", "consumers", "sums", "dz_ptr", "dz_ver",
                 "dz_shape")

    def __init__(self):
        self.consumers = 0
        self.sums = None
        self.dz_ptr = None
        self.dz_ver = None
        self.dz_shape = None
        self.x2 = self.y2 = self.mean = self.invstd = self.w32 = self.b32 = None

    def ready(self) -> bool:
        """A producer filled the slot: x2 (BN input, with y2 when a residual was
        fused), or y2 alone for a BN folded through its conv (ops/bn_fold.py):
        the consumer then reduces only sum dz."""
        return self.x2 is not None or self.y2 is not None

    def park(self, dz: torch.Tensor, sums: torch.Tensor) -> None:
        self.sums = sums
        self.dz_ptr, self.dz_ver, self.dz_shape = dz.data_ptr(), dz._version, tuple(dz.shape)

    def take(self, dy: torch.Tensor):
        sums, self.sums = self.sums, None
        if sums is None or dy.data_ptr() != self.dz_ptr or dy._version != self.dz_ver \
                or tuple(dy.shape) != self.dz_shape:
            return None
        return sums


_STATS["fused_bwd_moments"] = 0


# --------------------------------------------------------------------------- #
# Autograd function
# --------------------------------------------------------------------------- #
class _BatchNormActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, weight, bias, running_mean, running_var, training, momentum, eps,
                act_clip, reduce_moments, reduce_grads, pre_sums=None, nbt=None, bwd_slot=None,
                out_moments=False):
        relu = act_clip is not None
        clip = act_clip if relu else _INF
        x2, back = _as_rows(x)
        native = _native_ok(x2)
        _STATS["native_fwd" if native else "torch_fwd"] += 1
        if pre_sums is not None:
            _STATS["fused_moments"] = _STATS.get("fused_moments", 0) + 1
        res2 = None
        if residual is not None:
            res2, _ = _as_rows(residual.to(x.dtype))
        w32 = weight.float() if weight is not None else None
        b32 = bias.float() if bias is not None else None
        if training:
            # moments may come fused from the producing conv's epilogue (GEMM / depthwise)
            sums = pre_sums if pre_sums is not None else local_moments(x2, native)
            if reduce_moments is not None:
                sums = reduce_moments(sums)
            count = sums[-1:]
            upd_rm = running_mean if (running_mean is not None and running_mean.dtype == torch.float32) else None
            upd_rv = running_var if upd_rm is not None else None
            res = forward_apply(x2, sums, w32, b32, upd_rm, upd_rv, momentum, eps, res2, relu, native, nbt,
                                out_moments, clip)
            y2, mean, invstd = res[0], res[1], res[2]
            osums = res[3] if out_moments else None
            if running_mean is not None and upd_rm is None:  # low-precision buffers
                c = x2.shape[1]
                n = sums[2 * c]
                unbiased = (sums[c:2 * c] / n - mean.double() ** 2) * n / (n - 1).clamp_min(1)
                running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
                running_var.mul_(1 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
        else:
            count = torch.full((1,), float(x2.shape[0]), dtype=torch.float64, device=x2.device)
            y2, mean, invstd = eval_apply(x2, running_mean, running_var, w32, b32, eps, res2, relu,
                                          native, clip)
            osums = None
        # the ReLU mask needs the output only when a residual was added before the
        # ReLU; otherwise backward re-derives it from x (one tensor read fewer)
        ctx.save_for_backward(x2, y2 if (relu and residual is not None) else None, w32, b32, mean,
                              invstd, count)
        ctx.meta = (native, training, relu, residual is not None, back,
                    weight is not None, bias is not None, reduce_grads,
                    weight.dtype if weight is not None else None, x.dim(), clip)
        ctx.affine = (weight, bias)  # the leaves: micro-batch accumulation targets (ops/grad_accum.py)
        ctx.bwd_slot = None
        # the consumer-epilogue fusion applies a plain ReLU mask: not for ReLU6
        if bwd_slot is not None and native and training and relu and clip == _INF and x.dim() == 4:
            bwd_slot.x2 = x2
            bwd_slot.y2 = y2 if residual is not None else None
            bwd_slot.mean, bwd_slot.invstd, bwd_slot.w32, bwd_slot.b32 = mean, invstd, w32, b32
            ctx.bwd_slot = bwd_slot
        if out_moments:
            if osums is None:  # eval mode: moments of the output on request all the same
                yd = y2.double()
                osums = torch.cat([yd.sum(0), (yd * yd).sum(0), yd.new_tensor([float(y2.shape[0])])])
            ctx.mark_non_differentiable(osums)
            # osums never gets a gradient: no zero [2C+1] fp64 fill per backward
            ctx.set_materialize_grads(False)
            return back(y2), osums
        return back(y2)

    @staticmethod
    def backward(ctx, dy, _dosums=None):
        if dy is None:
            return (None,) * 16
        x2, y2, w32, b32, mean, invstd, count = ctx.saved_tensors
        (native, training, relu, has_res, back, has_w, has_b, reduce_grads, wdtype,
         ndim, clip) = ctx.meta
        dy2, _ = _as_rows(dy.to(x2.dtype))
        slot = ctx.bwd_slot
        fused = slot.take(dy) if slot is not None else None
        ctx.bwd_slot = None
        if fused is not None:
            # the consumer's dgrad epilogue already masked dy (dz) and reduced the moments
            _STATS["fused_bwd_moments"] += 1
            sums = fused
            relu_eff, y_eff, want_dres = False, None, False
        else:
            sums = backward_moments(dy2, x2, y2, mean, relu, native, w32, b32, invstd, clip)
            relu_eff, y_eff, want_dres = relu, y2, has_res
        local_sums = sums
        if training and reduce_grads is not None:
            local_sums = sums.clone()  # the reducer works in place
            sums = reduce_grads(sums)
        acc_w = acc_b = None
        if native and training and reduce_grads is None and has_w and has_b \
                and ctx.needs_input_grad[2] and ctx.needs_input_grad[3]:
            # micro-batch accumulation: the apply kernel adds the affine gradients
            # into weight.grad / bias.grad (fp32 parameters only)
            pw, pb = ctx.affine
            if pw.dtype == torch.float32 and pb.dtype == torch.float32:
                acc_w = grad_accum.target(pw)
                acc_b = grad_accum.target(pb) if acc_w is not None else None
                if acc_b is None:
                    acc_w = None
        ctx.affine = None
        dx2, dw, db, dres2 = backward_apply(dy2, x2, y_eff, sums, count, w32, mean, invstd, training,
                                            relu_eff, want_dres, native, b32, clip, acc_w, acc_b)
        if fused is not None and has_res:
            dres2 = dy2  # d(residual) = dz, which is exactly the masked incoming gradient
        if reduce_grads is not None and training:
            # weight/bias grads are per-rank quantities (DDP averages them)
            c = x2.shape[1]
            dw = (local_sums[c:] * invstd.double()).float()
            db = local_sums[:c].float()
        gx = back(dx2)
        gres = back(dres2) if has_res else None
        gw = dw.to(wdtype) if has_w and ctx.needs_input_grad[2] and acc_w is None else None
        gb = db.to(wdtype) if has_b and ctx.needs_input_grad[3] and acc_b is None else None
        return gx, gres, gw, gb, None, None, None, None, None, None, None, None, None, None, None, None


def batch_norm_act(x: torch.Tensor, running_mean: Optional[torch.Tensor],
                   running_var: Optional[torch.Tensor], weight: Optional[torch.Tensor],
                   bias: Optional[torch.Tensor], training: bool, momentum: float, eps: float,
                   relu: bool = False, residual: Optional[torch.Tensor] = None,
                   reduce_moments: Optional[MomentReducer] = None,
                   reduce_grads: Optional[GradReducer] = None,
                   sums: Optional[torch.Tensor] = None,
                   num_batches_tracked: Optional[torch.Tensor] = None,
                   out_moments: bool = False, act: Optional[str] = "_from_relu"):
    """Functional fused BN(+residual)(+ReLU).  `sums`: precomputed local moments
    [2C+1] of `x` (from a fused conv epilogue); ignored in eval mode.
    `num_batches_tracked`: incremented once (training mode), in-kernel when native.
    `out_moments`: also return the fp64 [2C+1] (colsum, colsum of squares, rows)
    of the OUTPUT, reduced inside the apply pass (ops/bn_fold.py needs colsum).
    `act`: None / "relu" / "relu6" (overrides `relu` when given)."""
    if act == "_from_relu":
        act = "relu" if relu else None
    if act not in ACTS:
        raise ValueError(f"unsupported activation {act!r}")
    clip = ACTS[act]
    slot = None
    if training and act == "relu" and x.dim() == 4 and torch.is_grad_enabled() and _FUSE_BWD \
            and _native.gpu_path(x):
        slot = BnBwdSlot()
    out = _BatchNormActFn.apply(x, residual, weight, bias, running_mean, running_var, training,
                                momentum, eps, clip, reduce_moments, reduce_grads, sums,
                                num_batches_tracked if training else None, slot, out_moments)
    osums = None
    if out_moments:
        out, osums = out
    if slot is not None and slot.x2 is not None:
        out._dmp_bnbwd = slot  # a native 1x1 conv consuming `out` may fuse our backward reductions
    return (out, osums) if out_moments else out


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with optional fused residual add and ReLU.

    ``forward(x, residual=None)`` computes ``act(bn(x) + residual)``; ``act`` is
    None, "relu" or "relu6" (ReLU clipped at 6, in the same kernels).
    """

    def __init__(self, num_features: int, eps: float = 1e-5, momentum: Optional[float] = 0.1,
                 affine: bool = True, track_running_stats: bool = True, act: Optional[str] = None,
                 device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device, dtype)
        if act not in ACTS:
            raise ValueError(f"unsupported activation {act!r}")
        self.act = act

    def _check_input_dim(self, x):
        if x.dim() not in (2, 3, 4):
            raise ValueError(f"expected 2D-4D input (got {x.dim()}D input)")

    def _momentum(self) -> float:
        if self.momentum is None:
            return 1.0 / float(self.num_batches_tracked) if self.num_batches_tracked is not None else 0.0
        return float(self.momentum)

    def _moment_reducers(self):
        return None, None

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                sums: Optional[torch.Tensor] = None, out_moments: bool = False):
        self._check_input_dim(x)
        use_batch = self.training or not self.track_running_stats
        recompute = in_recompute()  # activation-checkpoint recompute: no second stat update
        nbt = None
        if self.training and self.track_running_stats and self.num_batches_tracked is not None \
                and not recompute:
            if self.momentum is None:  # cumulative average needs the count now (host read)
                self.num_batches_tracked.add_(1)
            else:                      # counted inside the BN apply kernel
                nbt = self.num_batches_tracked
        momentum = self._momentum() if (self.training and self.track_running_stats) else 0.0
        if recompute:
            momentum = 0.0
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        rmom, rgrad = self._moment_reducers() if use_batch else (None, None)
        return batch_norm_act(x, rm if self.track_running_stats else None,
                              rv if self.track_running_stats else None, self.weight, self.bias,
                              use_batch, momentum, self.eps, act=self.act,
                              residual=residual, reduce_moments=rmom, reduce_grads=rgrad,
                              sums=sums if use_batch else None,
                              num_batches_tracked=nbt if use_batch else None,
                              out_moments=out_moments)

    def extra_repr(self) -> str:
        return super().extra_repr() + (f", act={self.act}" if self.act else "")


def reference_bn_act(x, rm, rv, w, b, training, momentum, eps, relu=False, residual=None, act=None):
    """Plain PyTorch composition used as the numerics oracle in tests."""
    y = F.batch_norm(x, rm, rv, w, b, training, momentum, eps)
    if residual is not None:
        y = y + residual
    if act == "relu6":
        return F.relu6(y)
    return F.relu(y) if (relu or act == "relu") else y
