"""Vision Transformer ViT-B/16 (86,567,656 parameters at 1000 classes, the
torchvision layout: conv patch embedding, class token, learned positional
embedding, 12 pre-LN encoder blocks, LayerNorm + linear head).

BASELINE.json config 5 ("ViT-B/16 DDP bf16 ... large-grad bucket fusion, MFMA
GEMM path").  The encoder is written so that all matmuls are plain GEMMs on
[B*T, D] activations (patch embedding, qkv, proj, fc1, fc2 and every data /
weight gradient run on the hand-written MFMA GEMMs of csrc/gemm/gemm_xl.hip) and
attention runs on the packed-qkv HIP kernels (ops/attention.py) with no
head split / merge copies; no per-head Python loops.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import self_attention_packed
from ..ops.fused import GradSlot, grad_tap
from ..ops.layernorm import LayerNorm
from ..ops.linear import Linear, linear_gelu, linear_residual, mlp_residual
from ..ops.patch_embed import PatchEmbed


class MLP(nn.Module):
    def __init__(self, dim: int, hidden: int, dropout: float = 0.0):
        super().__init__()
        self.fc1 = Linear(dim, hidden)
        self.fc2 = Linear(hidden, dim)
        self.dropout = dropout

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # fc1 + GELU: the backward fuses gelu'(h) with fc1's bias gradient (ops/linear.py)
        x = linear_gelu(x, self.fc1.weight, self.fc1.bias)
        x = F.dropout(x, self.dropout, self.training)
        return F.dropout(self.fc2(x), self.dropout, self.training)

    def forward_residual(self, x: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
        """res + forward(x) with the GELU and residual add inside the GEMM epilogues."""
        return mlp_residual(x, res, self.fc1, self.fc2, self.dropout, self.training)


class SelfAttention(nn.Module):
    def __init__(self, dim: int, heads: int, dropout: float = 0.0):
        super().__init__()
        assert dim % heads == 0
        self.heads = heads
        self.qkv = Linear(dim, 3 * dim)
        self.proj = Linear(dim, dim)
        self.dropout = dropout

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # packed-qkv attention (ops/attention.py): the fused HIP kernels read the
        # qkv GEMM output and write the proj GEMM input / the qkv gradient as is
        return self.proj(self._core(x))

    def _core(self, x: torch.Tensor) -> torch.Tensor:
        return self_attention_packed(self.qkv(x), self.heads, self.dropout if self.training else 0.0)

    def forward_residual(self, x: torch.Tensor, res: torch.Tensor) -> torch.Tensor:
        """res + forward(x): bias and residual added in the proj GEMM's store."""
        return linear_residual(self._core(x), res, self.proj.weight, self.proj.bias)


class EncoderBlock(nn.Module):
    def __init__(self, dim: int, heads: int, mlp_dim: int, dropout: float = 0.0):
        super().__init__()
        self.ln1 = LayerNorm(dim, eps=1e-6)
        self.attn = SelfAttention(dim, heads, dropout)
        self.ln2 = LayerNorm(dim, eps=1e-6)
        self.mlp = MLP(dim, mlp_dim, dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # pre-LN residuals: each LayerNorm's backward also adds the residual
        # branch's gradient of its input (ops/fused.py GradSlot) -- no add kernel.
        # The tap is created after the LN so its backward node runs first.
        train = self.training and torch.is_grad_enabled()
        s1 = GradSlot() if train else None
        h = self.ln1(x, s1)
        x = self.attn.forward_residual(h, grad_tap(x, s1))
        s2 = GradSlot() if train else None
        h = self.ln2(x, s2)
        return self.mlp.forward_residual(h, grad_tap(x, s2))


class VisionTransformer(nn.Module):
    def __init__(self, image_size: int = 224, patch_size: int = 16, num_layers: int = 12,
                 num_heads: int = 12, hidden_dim: int = 768, mlp_dim: int = 3072,
                 num_classes: int = 1000, dropout: float = 0.0):
        super().__init__()
        assert image_size % patch_size == 0
        self.patch_size = patch_size
        self.hidden_dim = hidden_dim
        # 16x16 / s16 conv as one MFMA GEMM over the patches (ops/patch_embed.py)
        self.patch_embed = PatchEmbed(3, hidden_dim, patch_size)
        n_tokens = (image_size // patch_size) ** 2 + 1
        self.cls_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.pos_embedding = nn.Parameter(torch.empty(1, n_tokens, hidden_dim).normal_(std=0.02))
        self.blocks = nn.Sequential(*[EncoderBlock(hidden_dim, num_heads, mlp_dim, dropout)
                                      for _ in range(num_layers)])
        self.ln = LayerNorm(hidden_dim, eps=1e-6)
        self.head = nn.Linear(hidden_dim, num_classes)
        self._init()

    def _init(self):
        fan_in = 3 * self.patch_size ** 2
        nn.init.trunc_normal_(self.patch_embed.weight, std=math.sqrt(1.0 / fan_in))
        nn.init.zeros_(self.patch_embed.bias)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)
        nn.init.zeros_(self.head.weight)
        nn.init.zeros_(self.head.bias)

    def tokens(self, x: torch.Tensor) -> torch.Tensor:
        x = self.patch_embed(x)  # [B, T, D]
        cls = self.cls_token.expand(x.shape[0], -1, -1).to(x.dtype)
        return torch.cat([cls, x], 1) + self.pos_embedding.to(x.dtype)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.blocks(self.tokens(x))
        return self.head(self.ln(x)[:, 0])


def vit_b_16(num_classes: int = 1000, image_size: int = 224, **kw) -> VisionTransformer:
    return VisionTransformer(image_size, 16, 12, 12, 768, 3072, num_classes, **kw)


def vit_tiny(num_classes: int = 10, image_size: int = 32, **kw) -> VisionTransformer:
    """Small config for CPU tests."""
    return VisionTransformer(image_size, 8, 2, 2, 32, 64, num_classes, **kw)
