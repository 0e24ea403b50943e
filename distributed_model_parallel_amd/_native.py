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


_PROBE = None  # utils/roofline.probe(): a timing proxy of the module (diagnostic only)


def native() -> Optional[ModuleType]:
    """The extension module, or None if it is not built/importable."""
    if _PROBE is not None:
        return _PROBE
    return _load()


def available() -> bool:
    return _load() is not None


def require(what: str = "this operation") -> ModuleType:
    """Return the extension or raise loudly (used on every GPU code path)."""
    if _PROBE is not None:
        return _PROBE
    m = _load()
    if m is None:
        raise RuntimeError(
            f"distributed_model_parallel_amd native extension is required for {what} but could "
            f"not be loaded ({_err!r}). Build it with `python csrc/build.py` "
            f"(or `python -c 'import __graft_entry__ as g; g.build()'`).")
    return m


# Native kernel paths / fusions that DMP_DISABLE=<name>[,<name>...] turns off
# (A/B measurement and bisection; the fallback is the unfused native path or
# the stock op).  The one kernel-selection switch of the framework.
FEATURES = {
    "igemm": "every native 3x3 conv (ops/conv_igemm.py) -> MIOpen",
    "halo3": "halo-tiled 3x3 convs of layers 1-2 (conv3x3_halo.hip, conv3x3_c128.hip)",
    "xl_conv3": "256x256 ping-pong implicit GEMM for layer-3/4 3x3 convs (gemm_xl.hip conv_xl)",
    "xl_conv": "256x256 ping-pong GEMM for wide 1x1 convs (gemm_xl.hip)",
    "tn_xl": "ping-pong TN weight gradients of wide 1x1 convs and of the ViT linears",
    "xl_linear": "ViT MLP / attention projection on the fused-epilogue ping-pong GEMM -> hipBLASLt + GELU / add passes",
    "compact_shortcut": "stride-2 shortcut gradient kept compact (no zero-filled tensor)",
    "fuse_bn_bwd": "BN backward reductions in the consumer's data-gradient epilogue (BnBwdSlot)",
    "fuse_stem_pool": "stem BN apply + ReLU inside the max-pool (forward and backward)",
    "stem_halo": "halo-tiled stem kernels (stem_halo.hip) -> row-tap implicit GEMM",
    "rowtap_stem": "row-tap stem implicit GEMM (stem.hip) -> MIOpen",
    "bn_fold": "bottleneck bn3 folded through conv3 (ops/bn_fold.py) -> conv + BN apply passes",
    "bn_fold_ds": "downsample conv + BN folded into the same GEMM as bn3 (ops/bn_fold.py) -> separate shortcut",
    "fuse_stem_wgrad": "stem BN backward apply folded into the stem weight gradient (ops/fused.py) "
                       "-> the apply pass + one weight gradient",
    "async_wgrad": "weight gradients on a side stream beside the data-gradient chain (ops/wgrad_stream.py) "
                   "-> inline on the compute stream",
}
_disabled_cache: Optional[frozenset] = None


def disabled(feature: str) -> bool:
    """True when ``feature`` (a FEATURES key) is listed in DMP_DISABLE."""
    global _disabled_cache
    if _disabled_cache is None:
        names = {f.strip() for f in os.environ.get("DMP_DISABLE", "").split(",") if f.strip()}
        unknown = names - set(FEATURES)
        if unknown:
            raise ValueError(f"DMP_DISABLE: unknown feature(s) {sorted(unknown)}; known: {sorted(FEATURES)}")
        _disabled_cache = frozenset(names)
    if feature not in FEATURES:
        raise KeyError(feature)
    return feature in _disabled_cache


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
