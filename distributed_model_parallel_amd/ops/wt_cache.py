"""Transposed weights (W^T) of the 1x1-conv data gradients, computed once per
weight update instead of once per backward use.

The data-gradient GEMM of a 1x1 conv reads W^T ([Cin, Cout], K-contiguous
rows for the MFMA kernel), so every backward ran ``w.t().contiguous()``: one
copy kernel per conv per backward (ResNet-50: ~50 per step; a MobileNetV2
pipeline micro-batch: ~35).  Two caches serve those operands:

* **Optimizer-driven (global).** A weight whose W^T a backward needed is
  noted.  After every step of our optimizers (``ops/optim.py`` FlatSGD /
  MasterSGD) :func:`after_optimizer_step` re-transposes every noted weight
  THAT OPTIMIZER OWNS in ONE launch (``_C.multi_transpose``) and stamps the
  entries with a generation and the weight's version counter.  Weights no
  optimizer of ours updates (e.g. captured DataParallel replicas, refreshed
  by raw copies) never get an entry.
  A backward then takes the buffer iff it was refreshed after the latest
  optimizer step and the weight has not been modified in place since (its
  ``_version``).  Our optimizers write through raw pointers, so they bump no
  version; any other in-place change does, and the op falls back to a fresh
  copy.  Buffers keep their storage, so captured steps (bench.py --graph)
  read them and the captured optimizer step refreshes them on every replay.
* **Per-step (pipeline).** :class:`WTCache` holds buffers for a stage's
  weights, refreshed by the pipeline before a step's first micro-batch.
  This covers any optimizer, since the pipeline itself refreshes.

Keyed by storage address and shape: a re-homed parameter misses until it is
registered again.
"""
from __future__ import annotations

import contextlib
import weakref
from typing import Dict, Iterable, Iterator, List, Optional, Tuple

import torch

_ACTIVE: list = [None]  # the per-step WTCache consulted first, or None
_STATS = {"hit": 0, "miss": 0, "refresh_launches": 0}
_GEN = [0]  # optimizer step generation

# key -> [weakref(weight), buf, generation, version]
_GLOBAL: Dict[Tuple[int, Tuple[int, ...]], list] = {}
_WANTED: set = set()  # keys a backward asked for that have no entry yet
_ENABLED = [True]


def _key(w: torch.Tensor) -> Tuple[int, Tuple[int, ...]]:
    return w.data_ptr(), tuple(w.shape)


def _native_transpose(srcs: List[torch.Tensor], dsts: List[torch.Tensor]) -> None:
    from .. import _native
    C = _native.native()
    if C is not None and srcs and srcs[0].is_cuda and hasattr(C, "multi_transpose") \
            and all(s.element_size() == 2 for s in srcs):
        C.multi_transpose(srcs, dsts)
        _STATS["refresh_launches"] += 1
        return
    for s, d in zip(srcs, dsts):
        d.copy_(s.t())


def set_enabled(on: bool) -> None:
    """Turn the optimizer-driven cache on / off (tests, A/B runs)."""
    _ENABLED[0] = bool(on)
    if not on:
        _GLOBAL.clear()
        _WANTED.clear()


def after_optimizer_step(params: Iterable[torch.Tensor] = ()) -> None:
    """Called by our optimizers after they updated ``params``: re-transpose
    every wanted weight among them in one launch and validate its entry;
    entries of freed or re-homed weights are dropped."""
    _GEN[0] += 1
    if not _ENABLED[0] or not (_GLOBAL or _WANTED):
        return
    srcs, dsts = [], []
    with torch.no_grad():
        for k in [k for k, e in _GLOBAL.items() if e[0]() is None or _key(e[0]()) != k]:
            del _GLOBAL[k]
        for p in params:
            if p.dim() not in (2, 4) or p.element_size() != 2:
                continue
            k = _key(p)
            e = _GLOBAL.get(k)
            if e is None and k in _WANTED:
                w2 = p.detach().reshape(p.shape[0], -1)
                e = _GLOBAL[k] = [weakref.ref(p), torch.empty(w2.shape[1], w2.shape[0], dtype=p.dtype,
                                                              device=p.device), -1, -1]
            if e is None or e[0]() is not p:
                continue
            srcs.append(p.detach().reshape(p.shape[0], -1))
            dsts.append(e[1])
            e[2], e[3] = _GEN[0], p._version
        _WANTED.clear()
        _native_transpose(srcs, dsts)


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
        """Re-register moved weights and transpose every W (once per step, one
        launch on the GPU)."""
        live = {}
        srcs, dsts = [], []
        with torch.no_grad():
            for p in self._params:
                k = _key(p)
                w2 = p.detach().reshape(p.shape[0], -1)
                buf = self._bufs.get(k)
                if buf is None or buf.dtype != p.dtype or buf.device != p.device:
                    buf = torch.empty(w2.shape[1], w2.shape[0], dtype=p.dtype, device=p.device)
                srcs.append(w2)
                dsts.append(buf)
                live[k] = buf
            _native_transpose(srcs, dsts)
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
    """``w.reshape(out, -1).t().contiguous()``, from a cache when one holds a
    current copy of this weight."""
    c = _ACTIVE[0]
    if c is not None:
        buf = c.get(w)
        if buf is not None:
            _STATS["hit"] += 1
            return buf
    if _ENABLED[0]:
        k = _key(w)
        e = _GLOBAL.get(k)
        if e is not None and e[2] == _GEN[0] and e[3] == w._version and e[0]() is not None:
            _STATS["hit"] += 1
            return e[1]
        if e is None and w.is_leaf and w.requires_grad and w.element_size() == 2:
            _WANTED.add(k)  # the owning optimizer's next step keeps a transposed copy
    _STATS["miss"] += 1
    return w.reshape(w.shape[0], -1).t().contiguous()


def stats() -> dict:
    return dict(_STATS)
