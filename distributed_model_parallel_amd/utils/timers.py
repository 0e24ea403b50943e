"""Timers: the reference uses host ``time.time()`` with no device
synchronisation (``utils.py:41-72``), which under-counts asynchronous GPU
work.  :class:`StepTimer` brackets regions with HIP events on the current
stream (device time, no sync until read) and keeps a host wall clock for the
data-wait part, mirroring the reference's batch_time / data_time split."""
from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class StepTimer:
    def __init__(self, device: Optional[torch.device] = None):
        self.cuda = device is not None and torch.device(device).type == "cuda"
        self.events: Dict[str, List] = {}
        self.host: Dict[str, List[float]] = {}

    @contextmanager
    def region(self, name: str):
        if self.cuda:
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            t = time.perf_counter()
            yield
            b.record()
            self.events.setdefault(name, []).append((a, b))
        else:
            t = time.perf_counter()
            yield
        self.host.setdefault(name, []).append(time.perf_counter() - t)

    def summary(self, reset: bool = True) -> Dict[str, float]:
        """Mean milliseconds per region (device time on GPU, host time otherwise)."""
        out: Dict[str, float] = {}
        if self.cuda and self.events:
            torch.cuda.synchronize()
            for k, evs in self.events.items():
                out[k] = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        for k, v in self.host.items():
            out.setdefault(k, 1e3 * sum(v) / len(v))
            out[f"{k}_host"] = 1e3 * sum(v) / len(v)
        if reset:
            self.events.clear()
            self.host.clear()
        return out
