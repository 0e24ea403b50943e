"""Multi-head self-attention on the packed qkv projection output, on our HIP
kernels (``csrc/attn/attention.hip``): forward and backward read qkv
[B*S, 3*H*64] and write o [B*S, H*64] / dqkv [B*S, 3*H*64] directly, so the
head split/permute copies, the output transpose and the dq/dk/dv
concatenation of the generic SDPA path disappear.  ViT-sized sequences
(S <= 256) with head dim 64; anything else (CPU, dropout, other shapes) runs
``F.scaled_dot_product_attention``."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import _native

_STATS = {"native": 0, "torch": 0}


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv2d, B, S, H, scale):
        C = _native.require("attention")
        o, lse = C.attention_forward(qkv2d, B, S, H, scale)
        ctx.save_for_backward(qkv2d, o, lse)
        ctx.dims = (B, S, H, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv2d, o, lse = ctx.saved_tensors
        B, S, H, scale = ctx.dims
        C = _native.require("attention backward")
        dqkv = C.attention_backward(do.contiguous(), qkv2d, o, lse, B, S, H, scale)
        return dqkv, None, None, None, None


def self_attention_packed(qkv: torch.Tensor, heads: int, dropout_p: float = 0.0) -> torch.Tensor:
    """qkv [B, S, 3*D] (torchvision layout: [q | k | v], each [heads, D/heads])
    -> attention output [B, S, D] (heads merged, ready for the output projection)."""
    b, s, d3 = qkv.shape
    d = d3 // 3
    hd = d // heads
    scale = 1.0 / math.sqrt(hd)
    C = _native.native() if _native.gpu_path(qkv) else None
    if (C is not None and dropout_p == 0.0 and qkv.dtype == torch.bfloat16 and hd == 64
            and C.attention_supported(s, hd)):
        _STATS["native"] += 1
        q2 = qkv.reshape(b * s, d3)
        if q2.stride(1) != 1 or q2.stride(0) % 8:
            q2 = q2.contiguous()
        return _AttnFn.apply(q2, b, s, heads, scale).view(b, s, d)
    _STATS["torch"] += 1
    q, k, v = qkv.view(b, s, 3, heads, hd).permute(2, 0, 3, 1, 4).unbind(0)
    o = F.scaled_dot_product_attention(q, k, v, dropout_p=dropout_p)
    return o.transpose(1, 2).reshape(b, s, d)
