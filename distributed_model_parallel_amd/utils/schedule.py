"""Learning-rate schedules of the reference recipe:
``CosineAnnealingLR(T_max=epochs)`` stepped per epoch plus
``pytorch_warmup.LinearWarmup(warmup_period=10)`` with ``dampen()`` -- the
latter package is not installed, so :class:`LinearWarmup` reimplements its
semantics: the scheduled lr is multiplied by ``min(1, (step+1)/period)``.

Reference defect 11 (T_max=90 while training 100 epochs) is avoided by
:func:`build_schedule` using the real epoch count.
"""
from __future__ import annotations

import math
import warnings
from typing import List, Optional

import torch


class LinearWarmup:
    """Multiplicative linear warm-up applied on top of another schedule.

    Usage (reference order): ``scheduler.step(); warmup.dampen()`` once per
    epoch (or per iteration).  ``dampen`` rescales every param group's lr by
    ``omega = min(1, (t+1)/warmup_period)`` where t counts dampen calls,
    starting with the first call at construction time (like pytorch_warmup).
    """

    def __init__(self, optimizer: torch.optim.Optimizer, warmup_period: int, last_step: int = -1):
        if warmup_period < 1:
            raise ValueError("warmup_period must be >= 1")
        self.optimizer = optimizer
        self.warmup_period = warmup_period
        self.last_step = last_step
        self.lrs: List[float] = [g["lr"] for g in optimizer.param_groups]
        self.dampen()

    def warmup_factor(self, step: int) -> float:
        return min(1.0, (step + 1) / self.warmup_period)

    def dampen(self, step: Optional[int] = None) -> None:
        if step is None:
            step = self.last_step + 1
        self.last_step = step
        omega = self.warmup_factor(step)
        self.lrs = [g["lr"] for g in self.optimizer.param_groups]  # undampened values
        for g in self.optimizer.param_groups:
            # the underlying scheduler has just written g["lr"]; scale it
            g["lr"] = g["lr"] * omega

    class _Dampening:
        def __init__(self, w: "LinearWarmup"):
            self.w = w

        def __enter__(self):
            for g, lr in zip(self.w.optimizer.param_groups, self.w.lrs):
                g["lr"] = lr  # let the wrapped scheduler see the undampened lr
            return self

        def __exit__(self, *exc):
            self.w.dampen()
            return False

    def dampening(self) -> "_Dampening":
        """``with warmup.dampening(): scheduler.step()`` -- exact for chainable schedulers."""
        return LinearWarmup._Dampening(self)

    def state_dict(self):
        return {"last_step": self.last_step, "warmup_period": self.warmup_period}

    def load_state_dict(self, sd):
        self.last_step = sd["last_step"]
        self.warmup_period = sd["warmup_period"]


def cosine_lr(base_lr: float, epoch: float, total: float, min_lr: float = 0.0) -> float:
    return min_lr + 0.5 * (base_lr - min_lr) * (1.0 + math.cos(math.pi * min(epoch, total) / total))


class WarmupCosine:
    """Closed-form per-epoch schedule: lr(e) = cosine(base, e, epochs) * min(1, (e+1)/warmup)."""

    def __init__(self, optimizer: torch.optim.Optimizer, epochs: int, warmup_epochs: int = 10,
                 min_lr: float = 0.0):
        self.optimizer = optimizer
        self.epochs = max(1, epochs)
        self.warmup = max(1, warmup_epochs)
        self.min_lr = min_lr
        self.base = [g.get("initial_lr", g["lr"]) for g in optimizer.param_groups]
        for g, b in zip(optimizer.param_groups, self.base):
            g["initial_lr"] = b
        self.epoch = 0
        self._apply()

    def _apply(self) -> None:
        w = min(1.0, (self.epoch + 1) / self.warmup)
        for g, b in zip(self.optimizer.param_groups, self.base):
            g["lr"] = cosine_lr(b, self.epoch, self.epochs, self.min_lr) * w

    def step(self, epoch: Optional[int] = None) -> None:
        self.epoch = self.epoch + 1 if epoch is None else epoch
        self._apply()

    def get_last_lr(self) -> List[float]:
        return [g["lr"] for g in self.optimizer.param_groups]

    kind = "cosine"

    def state_dict(self):
        return {"kind": self.kind, "epoch": self.epoch, "base": self.base, "epochs": self.epochs,
                "warmup": self.warmup}

    def _check_kind(self, sd) -> None:
        saved = sd.get("kind", "multistep" if "milestones" in sd else "cosine")
        if saved != self.kind:
            warnings.warn(f"resuming a {saved!r} lr schedule checkpoint with a {self.kind!r} schedule: "
                          f"the current command line's schedule type is kept", stacklevel=3)

    def load_state_dict(self, sd):
        self._check_kind(sd)
        self.epoch, self.base, self.epochs, self.warmup = sd["epoch"], sd["base"], sd["epochs"], sd["warmup"]
        self._apply()


class WarmupMultiStep(WarmupCosine):
    """Step decay: lr(e) = base * gamma^(number of milestones <= e) * min(1, (e+1)/warmup).

    The reference's no-BN large-batch study trains with "Linear decay (at
    30,60)" (Readme.md:170): the lr drops by ``gamma`` at epochs 30 and 60
    (torch ``MultiStepLR`` semantics, stepped per epoch)."""

    def __init__(self, optimizer: torch.optim.Optimizer, milestones, gamma: float = 0.1,
                 warmup_epochs: int = 0, epochs: int = 90):
        self.milestones = sorted(int(m) for m in milestones)
        self.gamma = float(gamma)
        super().__init__(optimizer, epochs, warmup_epochs)

    def _apply(self) -> None:
        w = min(1.0, (self.epoch + 1) / self.warmup)
        k = sum(1 for m in self.milestones if m <= self.epoch)
        for g, b in zip(self.optimizer.param_groups, self.base):
            g["lr"] = b * self.gamma ** k * w

    kind = "multistep"

    def state_dict(self):
        sd = super().state_dict()
        sd.update(milestones=self.milestones, gamma=self.gamma)
        return sd

    def load_state_dict(self, sd):
        # a resumed run continues the checkpoint's schedule; a cosine checkpoint
        # (no milestones) keeps the command line's, and any difference is said
        ms, gamma = sd.get("milestones", self.milestones), sd.get("gamma", self.gamma)
        ms = sorted(int(m) for m in ms)
        if "milestones" in sd and (ms != self.milestones or float(gamma) != self.gamma):
            warnings.warn(f"checkpoint lr milestones {ms} / gamma {gamma} differ from the command line's "
                          f"{self.milestones} / {self.gamma}: resuming with the checkpoint's", stacklevel=2)
        self.milestones, self.gamma = ms, float(gamma)
        super().load_state_dict(sd)


def build_schedule(optimizer: torch.optim.Optimizer, epochs: int, warmup_epochs: int = 10,
                   lr_steps: Optional[List[int]] = None, gamma: float = 0.1):
    """Cosine over `epochs` (not a mismatched T_max, defect 11) + linear warm-up,
    or step decay at ``lr_steps`` (epochs) by ``gamma`` + the same warm-up."""
    if lr_steps:
        return WarmupMultiStep(optimizer, lr_steps, gamma, warmup_epochs, epochs)
    return WarmupCosine(optimizer, epochs, warmup_epochs)
