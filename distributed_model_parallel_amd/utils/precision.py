"""Precision policy: bf16 compute weights, fp32 normalisation parameters.

Conv / Linear / embedding parameters are stored in bf16 (the flat optimizer
keeps fp32 master copies and momentum), so forward/backward never pay autocast
cast kernels and the DDP buckets (and their RCCL all-reduce bytes) are half
size.  BatchNorm parameters and running statistics stay fp32: the fused BN
kernel reads bf16 activations and fp32 per-channel coefficients.
"""
from __future__ import annotations

import torch
import torch.nn as nn

_NORM_TYPES = (nn.modules.batchnorm._BatchNorm, nn.GroupNorm)


def cast_model(model: nn.Module, dtype: torch.dtype = torch.bfloat16,
               keep_batchnorm_fp32: bool = True) -> nn.Module:
    for mod in model.modules():
        if keep_batchnorm_fp32 and isinstance(mod, _NORM_TYPES):
            continue
        for name, p in list(mod.named_parameters(recurse=False)):
            if p.is_floating_point():
                p.data = p.data.to(dtype)
        for name, b in list(mod.named_buffers(recurse=False)):
            if b.is_floating_point():
                setattr(mod, name, b.to(dtype))
    return model


def parse_dtype(s: str) -> torch.dtype:
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
            "float32": torch.float32, "fp16": torch.float16}[s]
