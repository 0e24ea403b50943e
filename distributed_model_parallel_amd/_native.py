"""Loader for the native extension ``_C`` (HIP kernels + RCCL + DDP reducer).

The extension is built in-tree by ``csrc/build.py`` (``__graft_entry__.build``).
On a machine with a GPU the native path is mandatory: every op that has a HIP
implementation raises if ``_C`` is missing instead of silently falling back to
PyTorch.  On a CPU-only machine (CI / gloo tests) the pure-PyTorch fallbacks
are used for the math, while the C++ Reducer still runs if ``_C`` imports.
"""
from __future__ import annotations

import contextlib
import os
import threading
from types import ModuleType
from typing import Optional

import torch

_lock = threading.Lock()
_mod: Optional[ModuleType] = None
_err: Optional[BaseException] = None
_tried = False


def _load() -> Optional[ModuleType]:
    global _mod, _err, _tried
    with _lock:
        if _tried:
            return _mod
        _tried = True
        if os.environ.get("DMP_DISABLE_NATIVE") == "1":
            _err = RuntimeError("DMP_DISABLE_NATIVE=1")
            return None
        try:
            so = os.environ.get("DMP_NATIVE_SO")
            if so:  # e.g. the host-ASan build (csrc/build.py --asan)
                import importlib.util
                import sys
                spec = importlib.util.spec_from_file_location(f"{__package__}._C", so)
                _mod = importlib.util.module_from_spec(spec)
                spec.loader.exec_module(_mod)
                sys.modules[f"{__package__}._C"] = _mod
                return _mod
            from . import _C  # type: ignore[attr-defined]
            _mod = _C
        except ImportError as e:  # pragma: no cover - depends on build state
            _err = e
            _mod = None
        return _mod


def native() -> Optional[ModuleType]:
    """The extension module, or None if it is not built/importable."""
    return _load()


def available() -> bool:
    return _load() is not None


def require(what: str = "this operation") -> ModuleType:
    """Return the extension or raise loudly (used on every GPU code path)."""
    m = _load()
    if m is None:
        raise RuntimeError(
            f"distributed_model_parallel_amd native extension is required for {what} but could "
            f"not be loaded ({_err!r}). Build it with `python csrc/build.py` "
            f"(or `python -c 'import __graft_entry__ as g; g.build()'`).")
    return m


_REFERENCE = False


@contextlib.contextmanager
def reference_mode():
    """Test oracle only: inside this block every op takes its stock-PyTorch
    path (F.conv2d / F.batch_norm / F.linear ...) even on GPU tensors, so the
    SAME model object can be trained as a plain-PyTorch reference on the same
    device (tests/test_gpu_convergence.py).  Not thread-safe; never used by
    the framework itself."""
    global _REFERENCE
    prev, _REFERENCE = _REFERENCE, True
    try:
        yield
    finally:
        _REFERENCE = prev


def gpu_path(t: torch.Tensor) -> bool:
    """True when `t` should take the HIP path: it lives on a GPU.

    GPU tensors never fall back: if the extension is missing this raises
    (``reference_mode`` aside).
    """
    if _REFERENCE:
        return False
    if t.is_cuda:
        require(f"GPU op on {t.device}")
        return True
    return False
