"""Top-k accuracy and running averages (reference ``utils.py:215-229``)."""
from __future__ import annotations

from typing import List, Sequence

import torch


@torch.no_grad()
def accuracy(output: torch.Tensor, target: torch.Tensor, topk: Sequence[int] = (1,)) -> List[torch.Tensor]:
    """Percentage of samples whose target is among the top-k predictions, per k.

    Returns 1-element tensors (like the reference) on the output's device; no
    host synchronisation happens here.
    """
    maxk = min(max(topk), output.shape[1])
    batch = target.size(0)
    pred = output.topk(maxk, 1, True, True).indices.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    return [correct[:min(k, maxk)].reshape(-1).float().sum(0, keepdim=True).mul_(100.0 / batch)
            for k in topk]


class AverageMeter:
    """Running mean of a scalar; accepts tensors without forcing a sync until read."""

    def __init__(self, name: str = ""):
        self.name = name
        self.reset()

    def reset(self) -> None:
        self.sum = 0.0
        self.count = 0
        self._pending = []

    def update(self, value, n: int = 1) -> None:
        if isinstance(value, torch.Tensor):
            self._pending.append((value.detach().reshape(-1)[0] * n, n))
        else:
            self.sum += float(value) * n
            self.count += n

    def _flush(self) -> None:
        if self._pending:
            vals = torch.stack([v for v, _ in self._pending]).double().sum().item()
            self.sum += vals
            self.count += sum(n for _, n in self._pending)
            self._pending = []

    @property
    def avg(self) -> float:
        self._flush()
        return self.sum / max(self.count, 1)
