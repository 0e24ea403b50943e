"""Transposed weights shared by the micro-batches of one pipeline step.

The data-gradient GEMM of a 1x1 conv reads W^T ([Cin, Cout], K-contiguous
rows for the MFMA kernel), so every backward ran ``w.t().contiguous()``: one
copy kernel per conv per micro-batch (MobileNetV2: ~35 per 64-image
micro-batch, ~280 per 8-micro-batch step).  The weights do not change between
the micro-batches of a step, so a :class:`WTCache` holds one persistent W^T
buffer per registered weight, refreshed once per step (:meth:`refresh`, before
the first micro-batch), and the ops read it through :func:`transposed` while
the cache is active.  The buffers keep their storage across refreshes, so
captured stage graphs (parallel/pipeline.py ``_StageGraphs``) read them too.

Keyed by the weight's storage address and shape: a re-homed parameter (e.g.
an optimizer flattening parameters) misses and takes the plain copy until
:meth:`refresh` re-registers it.
"""
from __future__ import annotations

import contextlib
from typing import Dict, Iterable, Iterator, Optional, Tuple

import torch

_ACTIVE: list = [None]  # the WTCache consulted by transposed(), or None
_STATS = {"hit": 0, "miss": 0}


def _key(w: torch.Tensor) -> Tuple[int, Tuple[int, ...]]:
    return w.data_ptr(), tuple(w.shape)


class WTCache:
    def __init__(self, params: Iterable[torch.Tensor] = ()):
        self._params = []
        self._bufs: Dict[Tuple[int, Tuple[int, ...]], torch.Tensor] = {}
        for p in params:
            self.add(p)

    def add(self, p: torch.Tensor) -> None:
        if p.dim() not in (2, 4) or (p.dim() == 4 and p.shape[2:] != (1, 1)):
            return
        self._params.append(p)

    def refresh(self) -> None:
        """Re-register moved weights and copy every W^T (once per step)."""
        live = {}
        with torch.no_grad():
            for p in self._params:
                k = _key(p)
                w2 = p.detach().reshape(p.shape[0], -1)
                buf = self._bufs.get(k)
                if buf is None or buf.dtype != p.dtype or buf.device != p.device:
                    buf = torch.empty(w2.shape[1], w2.shape[0], dtype=p.dtype, device=p.device)
                buf.copy_(w2.t())
                live[k] = buf
        self._bufs = live

    def get(self, w: torch.Tensor) -> Optional[torch.Tensor]:
        return self._bufs.get(_key(w))

    @contextlib.contextmanager
    def active(self) -> Iterator[None]:
        prev = _ACTIVE[0]
        _ACTIVE[0] = self
        try:
            yield
        finally:
            _ACTIVE[0] = prev

    def __len__(self) -> int:
        return len(self._params)


def transposed(w: torch.Tensor) -> torch.Tensor:
    """``w.reshape(out, -1).t().contiguous()``, from the active cache when it
    holds this weight."""
    c = _ACTIVE[0]
    if c is not None:
        buf = c.get(w)
        if buf is not None:
            _STATS["hit"] += 1
            return buf
    _STATS["miss"] += 1
    return w.reshape(w.shape[0], -1).t().contiguous()


def stats() -> dict:
    return dict(_STATS)
