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
* **Flipped kh x kw weights (optimizer-driven).** The data gradient of a
  stride-1 kh x kw conv is the same conv over the flipped, transposed weight
  ``w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, -1)`` (conv_igemm: two
  torch kernels per 3x3 per backward, 13 per ResNet-50 step).  :func:`flipped`
  keeps it in the same cache (key kind ``"flip"``) and the optimizer's
  refresh forms it tap by tap in the same single ``multi_transpose`` launch.
  Channels-last weights only (their [Cout][kh][kw][Cin] storage is the
  [Cout, T*Cin] matrix the tap-wise transpose reads).
* **fp32 copies (optimizer-driven).** The BN-fold coefficient product reads
  the conv weight in fp32 (ops/bn_fold.py, one cast kernel per folded layer
  per forward); :func:`as_f32` keeps that cast (key kind ``"f32"``),
  refreshed by one ``multi_cast_bf16_f32`` launch per step.
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
_GLOBAL: Dict[tuple, list] = {}
_WANTED: set = set()  # keys a backward asked for that have no entry yet
_ENABLED = [True]
_FLIP = [True]  # flipped kh x kw entries (tools/step_ab.py arms flipc / flipt)


def _key(w: torch.Tensor, kind: str = "t") -> tuple:
    return (w.data_ptr(), tuple(w.shape)) if kind == "t" else (w.data_ptr(), tuple(w.shape), kind)


def _flip_src(p: torch.Tensor) -> Optional[torch.Tensor]:
    """The [Cout, T*Cin] storage view of a channels-last kh x kw weight, or None."""
    if p.dim() != 4 or not p.is_contiguous(memory_format=torch.channels_last):
        return None
    return p.detach().permute(0, 2, 3, 1).reshape(p.shape[0], -1)


def _native_transpose(srcs: List[torch.Tensor], dsts: List[torch.Tensor], taps: Optional[List[int]] = None) -> None:
    """dst = src^T; taps[i] = T (-T: flipped) transposes [R, T*C] -> [C, T*R] tap by tap."""
    from .. import _native
    taps = taps or [1] * len(srcs)
    C = _native.native()
    if C is not None and srcs and srcs[0].is_cuda and hasattr(C, "multi_transpose") \
            and all(s.element_size() == 2 for s in srcs):
        C.multi_transpose(srcs, dsts, taps)
        _STATS["refresh_launches"] += 1
        return
    for s, d, tp in zip(srcs, dsts, taps):
        T = abs(tp)
        r, c = s.shape[0], s.shape[1] // T
        blk = s.reshape(r, T, c)
        if tp < 0:
            blk = blk.flip(1)
        d.copy_(blk.permute(2, 1, 0).reshape(c, T * r))


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
    params = list(params)  # walked twice (transposes, then casts)
    srcs, dsts, taps = [], [], []
    with torch.no_grad():
        for k in [k for k, e in _GLOBAL.items()
                  if e[0]() is None or _key(e[0](), k[2] if len(k) > 2 else "t") != k]:
            del _GLOBAL[k]
        for p in params:
            if p.dim() not in (2, 4) or p.element_size() != 2:
                continue
            for kind in ("t", "flip"):
                k = _key(p, kind)
                e = _GLOBAL.get(k)
                if e is None and k not in _WANTED:
                    continue  # (no source view either: reshaping a channels-last 3x3 weight copies it)
                if kind == "t":
                    src, tp = p.detach().reshape(p.shape[0], -1), 1
                else:
                    src, tp = _flip_src(p), -(p.shape[2] * p.shape[3])
                    if src is None:  # no longer channels-last: drop the entry
                        _GLOBAL.pop(k, None)
                        continue
                if e is None and k in _WANTED:
                    T = abs(tp)
                    e = _GLOBAL[k] = [weakref.ref(p), torch.empty(src.shape[1] // T, src.shape[0] * T,
                                                                  dtype=p.dtype, device=p.device), -1, -1]
                if e is None or e[0]() is not p:
                    continue
                srcs.append(src)
                dsts.append(e[1])
                taps.append(tp)
                e[2], e[3] = _GEN[0], p._version
        csrc, cdst = [], []
        for p in params:
            if p.element_size() != 2 or p.dtype != torch.bfloat16:
                continue
            k = _key(p, "f32")
            e = _GLOBAL.get(k)
            if e is None and k in _WANTED:
                e = _GLOBAL[k] = [weakref.ref(p), torch.empty(p.shape[0], p.numel() // max(1, p.shape[0]),
                                                              dtype=torch.float32, device=p.device), -1, -1]
            if e is None or e[0]() is not p:
                continue
            csrc.append(p.detach().reshape(p.shape[0], -1))
            cdst.append(e[1])
            e[2], e[3] = _GEN[0], p._version
        _WANTED.clear()
        _native_transpose(srcs, dsts, taps)
        _native_cast(csrc, cdst)


def _native_cast(srcs: List[torch.Tensor], dsts: List[torch.Tensor]) -> None:
    if not srcs:
        return
    from .. import _native
    C = _native.native()
    if C is not None and srcs[0].is_cuda and hasattr(C, "multi_cast_bf16_f32") \
            and all(s.is_contiguous() for s in srcs):
        C.multi_cast_bf16_f32(srcs, dsts)
        _STATS["refresh_launches"] += 1
        return
    for s, d in zip(srcs, dsts):
        d.copy_(s)


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


def flipped(w: torch.Tensor) -> torch.Tensor:
    """``w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, -1).contiguous()`` (the
    data-gradient weight of a stride-1 kh x kw conv), from the optimizer-driven
    cache when it holds a current copy of this weight."""
    if _ENABLED[0] and _FLIP[0] and w.dim() == 4:
        k = _key(w, "flip")
        e = _GLOBAL.get(k)
        if e is not None and e[2] == _GEN[0] and e[3] == w._version and e[0]() is not None:
            _STATS["hit"] += 1
            return e[1]
        if e is None and w.is_leaf and w.requires_grad and w.element_size() == 2 and \
                w.is_contiguous(memory_format=torch.channels_last):
            _WANTED.add(k)
    _STATS["miss"] += 1
    return w.flip(2, 3).permute(1, 2, 3, 0).reshape(w.shape[1], -1).contiguous()


def as_f32(w: torch.Tensor) -> Optional[torch.Tensor]:
    """fp32 copy [out, in] of a bf16 weight parameter from the optimizer-driven
    cache, or None (the caller casts) -- and then noted for the next refresh."""
    if not _ENABLED[0] or w.dtype != torch.bfloat16:
        return None
    k = _key(w, "f32")
    e = _GLOBAL.get(k)
    if e is not None and e[2] == _GEN[0] and e[3] == w._version and e[0]() is not None:
        _STATS["hit"] += 1
        return e[1]
    if e is None and w.is_leaf and w.requires_grad:
        _WANTED.add(k)
    _STATS["miss"] += 1
    return None


def stats() -> dict:
    return dict(_STATS)
