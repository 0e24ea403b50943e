"""conv -> BatchNorm(+residual)(+ReLU) with the BN statistics produced by the
conv kernel's epilogue when both run natively (1x1 MFMA GEMM or depthwise
3x3); otherwise the plain two-module path.  In training this removes the BN
moments pass over the conv output (one full HBM read per layer)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .batchnorm import BatchNormAct2d


def conv_bn(conv: nn.Module, bn: nn.Module, x: torch.Tensor,
            residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    fused = (isinstance(bn, BatchNormAct2d) and bn.training and hasattr(conv, "forward_with_moments"))
    if fused:
        y, sums = conv.forward_with_moments(x)
        return bn(y, residual, sums=sums)
    y = conv(x)
    if isinstance(bn, BatchNormAct2d):
        return bn(y, residual)
    if residual is not None:
        return bn(y) + residual
    return bn(y)
