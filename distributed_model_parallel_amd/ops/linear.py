"""Linear layers for the ViT encoder with native backward side passes
(``csrc/linear/bias_act.hip``).

* ``Linear``: drop-in ``nn.Linear``.  Forward is one library GEMM with the bias
  in its epilogue (``addmm`` -> hipBLASLt ``Bias`` kernels).  Backward runs the
  data-gradient library GEMM, the weight gradient on our ping-pong TN kernel
  (``_wgrad``) and takes the bias gradient with our column-sum
  kernel instead of PyTorch's generic reduce (1.77 ms -> see
  ``profiles/vit_b16_bs128_1gpu_v3.md``).
* ``linear_gelu``: fc1 + exact GELU; the backward fuses gelu'(h) with fc1's
  bias gradient in one pass over the pre-activation.

* ``mlp_residual`` / ``linear_residual``: the ViT block's MLP and attention
  output projection with the residual add, on our 256x256 ping-pong MFMA GEMM
  (``csrc/gemm/gemm_xl.hip``, PIPE 7) and its fused epilogues: fc1 writes the
  pre-activation and GELU(h) in one pass (no GELU kernel), fc2 / proj add bias
  and residual in the store (no add kernel), and fc2's data gradient applies
  gelu'(h) in its epilogue (no GELU-backward pass).  On by default since the
  weight gradients moved to the TN kernel: ViT-B/16 batch 256, 43.6 vs 43.7 ms
  per step in round 3 (tools/vit_step_ab.py, profiles/raw_r3/vit_step_ab.log;
  round 2 measured it 1.6 % slower with the library weight gradients,
  profiles/vit_xl_epilogues_r2.md).  ``DMP_DISABLE=xl_linear`` or
  ``set_xl_linear(False)`` selects hipBLASLt + the separate passes.

CPU tensors, non-bf16 dtypes and widths that are not a multiple of 256 use
the plain PyTorch ops (same math)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _native
from . import wgrad_stream

_STATS = {"native": 0, "torch": 0, "xl": 0, "tn_wgrad": 0, "xl_dgrad": 0, "xl_fwd": 0}
_XL = not _native.disabled("xl_linear")


def set_xl_linear(on: bool) -> None:
    """Route mlp_residual / linear_residual to the fused gemm_xl path."""
    global _XL
    _XL = bool(on)

_XL_MIN_ROWS = 4096  # below this the 256-row tile grid leaves most CUs idle
# The PLAIN GEMMs -- nothing to fuse but a bias: the qkv projection forward
# and the data gradients of qkv / proj / fc1 -- on hipBLASLt ("lib"), gemm_xl
# ("xl") or split ("fwd", the default, below).  The 4-wave kernel (gemm_xl PIPE 11, finding 69) ties the
# library in isolation on the N >= 2304 shapes (1.03-1.07 PF/s,
# tools/pipe_bench.py), but in the step the data gradients are all N = 768
# (591 tiles = 2.3 rounds of 256 CUs; the library's 256 x 224 tile fills them
# better) and need a W^T copy: 8.0 + 0.4 ms vs 7.4 ms per step (ViT 41.0 vs
# 40.3 ms).  The fused-epilogue GEMMs and every weight gradient (gemm_tn_xl)
# are ours.
# "fwd": the qkv forward (N = 2304, bias in the store) on ours, the N = 768
# data gradients on the library -- ViT step 36.56 / 36.67 ms (fwd) vs 36.55 /
# 36.61 (lib) vs 37.27 / 37.41 (xl), interleaved on one box, with 256-row
# tiles and a W^T copy per data gradient.
# "xl" (default since the 224-row tiles and the optimizer-driven W^T cache):
# the N = 768 grids fill their three rounds (678 tiles of 224 rows), and the
# data gradients tie the library in isolation (qkv / proj / fc1: 0.169 /
# 0.068 / 0.221 vs 0.165 / 0.070 / 0.221 ms, tools/w4_trim_bench.py) and in
# the step (tools/step_ab.py: xl 38.23 vs fwd 38.21 vs lib 38.05 ms on one
# box): no library GEMM left in the ViT step but the classifier head.
_PLAIN_MODE = __import__("os").environ.get("DMP_LINEAR_PLAIN", "xl")
_PLAIN_LIB = _PLAIN_MODE == "lib"
_PLAIN_FWD_XL = _PLAIN_MODE in ("xl", "fwd")
_PLAIN_DGRAD_XL = _PLAIN_MODE == "xl"


def _native_ok(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor]) -> bool:
    if not _native.gpu_path(x):
        return False
    C = _native.native()
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and b is not None
            and b.dtype == torch.bfloat16 and C.colsum_supported(w.shape[0]))


# Weight gradients dW = dy^T x on the ping-pong TN kernel (gemm_tn_xl: 256x256
# tiles, split over the token rows, one reduce): the ViT shapes have a tiny
# output (<= 3072 x 768) over a 50k-row reduction, where hipBLASLt's picks run at
# 340-650 TF/s (profiles/vit_b16_bs256_1gpu_lib_r2.md) -- tools/vit_wgrad_bench.py
_TN_WGRAD = not _native.disabled("tn_xl")
_TN_MIN_ROWS = 16384


def _gemm_operand_ok(t: torch.Tensor) -> bool:
    """What csrc/gemm/gemm_xl.hip check_bf16_2d demands of a GEMM operand:
    2-D bf16, unit column stride, 16-B aligned rows and base (a column-sliced
    or offset view fails here and takes the library path instead of raising
    in the kernel's TORCH_CHECK)."""
    return (t.dim() == 2 and t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.stride(0) % 8 == 0
            and t.data_ptr() % 16 == 0)


def _wgrad(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    # on the weight-gradient side stream, beside the data-gradient chain (ops/wgrad_stream.py)
    with wgrad_stream.side(w, dy2, x2):
        if (_TN_WGRAD and dy2.shape[0] >= _TN_MIN_ROWS and dy2.shape[1] >= 256 and x2.shape[1] >= 256
                and dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0 and _gemm_operand_ok(dy2)
                and _gemm_operand_ok(x2) and w.dtype == torch.bfloat16):
            _STATS["tn_wgrad"] += 1
            return _native.native().gemm_tn_xl(dy2, x2, w.dtype)
        return dy2.t().mm(x2)


def _xl_gemm_ok(a: torch.Tensor, n: int) -> bool:
    """C[M, n] = a @ B^T on gemm_xl: bf16 operand contract, K % 64, n % 64,
    and enough rows to fill the 256-row tile grid."""
    return (_XL and a.is_cuda and _native.native() is not None and a.shape[0] >= _XL_MIN_ROWS
            and a.shape[1] % 64 == 0 and n % 64 == 0 and _gemm_operand_ok(a))


def _dgrad(dy2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dx = dy @ W on gemm_xl (B operand = W^T [in, out], from the
    optimizer-driven W^T cache, ops/wt_cache.py), or hipBLASLt with
    DMP_LINEAR_PLAIN=lib / fwd."""
    if _PLAIN_DGRAD_XL and w.dtype == torch.bfloat16 and _xl_gemm_ok(dy2, w.shape[1]):
        _STATS["xl_dgrad"] += 1
        from .wt_cache import transposed
        return _native.native().gemm_xl(dy2, transposed(w))
    return dy2.mm(w)


def _weight_grads(ctx, dy2, x2, w):
    dx = _dgrad(dy2, w) if ctx.needs_input_grad[0] else None
    dw = _wgrad(dy2, x2, w) if ctx.needs_input_grad[1] else None
    return dx, dw


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        if _PLAIN_FWD_XL and _xl_gemm_ok(x2, w.shape[0]):  # the qkv projection: bias in the MFMA GEMM's store
            _STATS["xl_fwd"] += 1
            y = _native.native().gemm_xl(x2, w, "bias", bias=b)
        else:
            y = torch.addmm(b, x2, w.t())
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        C = _native.require("linear backward")
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        dx, dw = _weight_grads(ctx, dy2, x2, w)
        db = C.bias_grad(dy2, w.dtype) if ctx.needs_input_grad[2] else None
        return (dx.view(ctx.xshape) if dx is not None else None), dw, db


class _LinearGeluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1])
        h = torch.addmm(b, x2, w.t())
        ctx.save_for_backward(x2, w, h)
        ctx.xshape = x.shape
        return F.gelu(h).view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, da):
        x2, w, h = ctx.saved_tensors
        C = _native.require("linear+gelu backward")
        dh, db = C.gelu_bwd_bias_grad(da.reshape(h.shape).contiguous(), h, w.dtype)
        dx, dw = _weight_grads(ctx, dh, x2, w)
        return (dx.view(ctx.xshape) if dx is not None else None), dw, \
            (db if ctx.needs_input_grad[2] else None)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    if _native_ok(x, weight, bias):
        _STATS["native"] += 1
        return _LinearFn.apply(x, weight, bias)
    _STATS["torch"] += 1
    return F.linear(x, weight, bias)


def linear_gelu(x: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor]) -> torch.Tensor:
    """gelu(x @ W^T + b) (exact erf GELU, as ``nn.GELU()``)."""
    if _native_ok(x, weight, bias):
        _STATS["native"] += 1
        return _LinearGeluFn.apply(x, weight, bias)
    _STATS["torch"] += 1
    return F.gelu(F.linear(x, weight, bias))


class Linear(nn.Linear):
    """Drop-in ``nn.Linear`` whose backward uses the native bias-gradient kernel."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return linear(x, self.weight, self.bias)


# --------------------------------------------------------------------------- #
# Fused-epilogue paths on the ping-pong GEMM (ViT encoder block)
# --------------------------------------------------------------------------- #
def _xl_ok(x: torch.Tensor, *ws: torch.Tensor) -> bool:
    if not (_XL and _native.gpu_path(x)) or x.dtype != torch.bfloat16:
        return False
    C = _native.native()
    rows = x.numel() // x.shape[-1]
    return (rows >= _XL_MIN_ROWS and all(w.dtype == torch.bfloat16 and w.shape[1] % 64 == 0 and
                                         w.shape[0] % 64 == 0 and C.colsum_supported(w.shape[0]) for w in ws))


def _rows(t: torch.Tensor) -> torch.Tensor:
    t2 = t.reshape(-1, t.shape[-1])
    return t2 if t2.stride(-1) == 1 and t2.stride(0) % 8 == 0 else t2.contiguous()


class _LinearResidualFn(torch.autograd.Function):
    """y = res + (x @ W^T + b): bias and residual added in the GEMM's store."""

    @staticmethod
    def forward(ctx, x, res, w, b):
        C = _native.require("linear_residual")
        x2, r2 = _rows(x), _rows(res)
        y = C.gemm_xl(x2, w, "bias_res", bias=b, residual=r2)
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        C = _native.require("linear_residual backward")
        dy2 = _rows(dy)
        dx = _dgrad(dy2, w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = _wgrad(dy2, x2, w) if ctx.needs_input_grad[2] else None
        db = C.bias_grad(dy2, w.dtype) if ctx.needs_input_grad[3] else None
        return dx, dy, dw, db


class _MLPResidualFn(torch.autograd.Function):
    """y = res + fc2(gelu(fc1(x))) on three fused-epilogue GEMMs:
    fc1 -> (h, gelu(h)); fc2 -> bias + residual; fc2 dgrad -> * gelu'(h)."""

    @staticmethod
    def forward(ctx, x, res, w1, b1, w2, b2):
        C = _native.require("mlp_residual")
        x2, r2 = _rows(x), _rows(res)
        h = torch.empty(x2.shape[0], w1.shape[0], dtype=x2.dtype, device=x2.device)
        a = C.gemm_xl(x2, w1, "bias_gelu", bias=b1, aux=h)
        y = C.gemm_xl(a, w2, "bias_res", bias=b2, residual=r2)
        ctx.save_for_backward(x2, w1, h, a, w2)
        ctx.xshape = x.shape
        return y.view(res.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, w1, h, a, w2 = ctx.saved_tensors
        C = _native.require("mlp_residual backward")
        dy2 = _rows(dy)
        db2 = C.bias_grad(dy2, w2.dtype)
        dw2 = _wgrad(dy2, a, w2)
        # dh = bf16(bf16(dy @ W2) * gelu'(h)): B operand is W2^T [hidden, dim]
        # and fc1's bias gradient (column sums of dh) from the same epilogue
        from .wt_cache import transposed
        dh, db1 = C.gemm_xl_dgelu_bgrad(dy2, transposed(w2), h)
        db1 = db1.to(w1.dtype)
        dw1 = _wgrad(dh, x2, w1)
        dx = _dgrad(dh, w1)
        return dx.view(ctx.xshape), dy, dw1, db1, dw2, db2


def linear_residual(x: torch.Tensor, res: torch.Tensor, weight: torch.Tensor,
                    bias: torch.Tensor) -> torch.Tensor:
    """res + linear(x): one GEMM with the bias and residual in its epilogue."""
    if (bias is not None and bias.dtype == torch.bfloat16 and _xl_ok(x, weight)
            and res.dtype == torch.bfloat16 and res.shape[:-1] == x.shape[:-1]):
        _STATS["xl"] += 1
        return _LinearResidualFn.apply(x, res, weight, bias)
    return res + linear(x, weight, bias)


def mlp_residual(x: torch.Tensor, res: torch.Tensor, fc1: nn.Linear, fc2: nn.Linear,
                 dropout: float = 0.0, training: bool = False) -> torch.Tensor:
    """res + fc2(gelu(fc1(x))) (exact erf GELU, as ``nn.GELU()``)."""
    if ((dropout == 0.0 or not training) and fc1.bias is not None and fc2.bias is not None
            and fc1.bias.dtype == torch.bfloat16 and fc2.bias.dtype == torch.bfloat16
            and _xl_ok(x, fc1.weight, fc2.weight) and res.dtype == torch.bfloat16):
        _STATS["xl"] += 1
        return _MLPResidualFn.apply(x, res, fc1.weight, fc1.bias, fc2.weight, fc2.bias)
    hdn = F.dropout(linear_gelu(x, fc1.weight, fc1.bias), dropout, training)
    return res + F.dropout(linear(hdn, fc2.weight, fc2.bias), dropout, training)
