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
    """Per-forward-call mailbox between a grad_tap and one native consumer."""
    __slots__ = ("consumer", "consumer_ran", "grad")

    def __init__(self):
        self.consumer = False      # a native conv registered to absorb the parked grad
        self.consumer_ran = False  # its backward already ran without a parked grad
        self.grad: Optional[torch.Tensor] = None

    def take(self) -> Optional[torch.Tensor]:
        g, self.grad = self.grad, None
        if g is None:
            self.consumer_ran = True
        return g


class _GradTap(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
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
    return _GradTap.apply(x, slot)


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
