"""Whole-training-step hipGraph capture.

A ResNet-50 step is ~1000 kernel launches; eager PyTorch spends tens of
microseconds of host time per launch (Python, dispatcher, MIOpen solution
lookup), which on MI355X is comparable to the GPU time of the step.  The
MI355X-first answer is to capture the step once -- forward, backward with the
C++ reducer's RCCL all-reduces on the side stream (joined into the capture by
event edges), the fused flat optimizer -- and replay it as one hipGraph.

Constraints (checked by the caller): static input buffers (copy new data into
``inputs`` before each replay), no host synchronisation inside the step, and
the first optimizer step and DDP bucket rebuild must already have happened
(they run in the eager warm-up iterations).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    """Callable training step: the first ``warmup`` calls run eagerly (on a side
    stream, as capture requires), the next call captures the step into a
    hipGraph and replays it; every later call is one replay.  Each call advances
    the training state by exactly one step and returns the (static) loss."""

    def __init__(self, step_fn: Callable[[], torch.Tensor], warmup: int = 3,
                 comm_sync: Optional[Callable[[], None]] = None,
                 stream: Optional[torch.cuda.Stream] = None):
        self.step_fn = step_fn
        self.warmup = max(1, warmup)
        self.comm_sync = comm_sync
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.static_out: Optional[torch.Tensor] = None
        self._calls = 0
        self._side = stream  # warm-up and capture stream (the model/DDP should be built on it)

    def _eager(self) -> torch.Tensor:
        if self._side is None:
            self._side = torch.cuda.Stream()
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side):
            out = self.step_fn()
        torch.cuda.current_stream().wait_stream(self._side)
        return out

    def capture(self) -> None:
        if self._side is None:
            self._side = torch.cuda.Stream()
        torch.cuda.synchronize()
        if self.comm_sync is not None:
            self.comm_sync()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self._side):
            out = self.step_fn()
        torch.cuda.synchronize()
        self.graph = g
        self.static_out = out

    def __call__(self) -> torch.Tensor:
        self._calls += 1
        if self._calls <= self.warmup:
            return self._eager()
        if self.graph is None:
            self.capture()  # records only; the replay below executes the step
        self.graph.replay()
        return self.static_out
