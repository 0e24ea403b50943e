"""Per-call roofline probe of the native extension (diagnostic, tools/step_roofline.py).

While active, every function of ``_C`` that the ops call is timed in
isolation (device synchronize, HIP events around the call, synchronize) and
priced: FLOPs from the operand shapes for the GEMM / convolution / attention
entry points, bytes = every tensor operand read once + every tensor result
written once (a lower bound on the HBM traffic: tile re-reads, fp32 split
partials and scratch are not counted).  The roofline bound of a call is
max(FLOPs / 2.5 PF/s, bytes / 8 TB/s) -- MI355X dense bf16 MFMA and HBM3E
peaks (MI355X_MICROARCH.md); its achieved fraction is bound / measured time.

Only the _C entry points are seen: library kernels (MIOpen, hipBLASLt) and
torch elementwise ops appear as the difference between the plain step time
and the sum of the probed calls.
"""
from __future__ import annotations

import contextlib
from typing import Any, Dict, List

import torch

PEAK_FLOPS = 2.5e15
PEAK_BYTES = 8.0e12


def _tensors(x) -> List[torch.Tensor]:
    if isinstance(x, torch.Tensor):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for v in x for t in _tensors(v)]
    return []


def _nbytes(ts) -> int:
    return sum(t.numel() * t.element_size() for t in ts if t.is_cuda)


def _arg(args, kw, i, name, default=None):
    if len(args) > i:
        return args[i]
    return kw.get(name, default)


def _rows4(x: torch.Tensor) -> int:
    """Pixels of a 4-D NCHW/NHWC tensor or rows of a 2-D one."""
    return x.shape[0] * x.shape[2] * x.shape[3] if x.dim() == 4 else x.shape[0]


def flops(name: str, args, kw) -> float:
    a0 = args[0] if args else None
    try:
        if name in ("gemm_nt", "gemm_nt_bnbwd", "gemm_xl", "gemm_xl_conv", "gemm_xl_dgelu_bgrad"):
            B = args[1]
            return 2.0 * a0.shape[0] * B.shape[0] * B.shape[1]
        if name in ("gemm_tn", "gemm_tn_xl"):
            B = args[1]
            m = a0.shape[0]
            bmap = _arg(args, kw, 3, "b_map", [])
            if bmap and _arg(args, kw, 6, "a_mapped", False):
                s, ho, wo, hi, wi = bmap
                m = m // (hi * wi) * ho * wo
            return 2.0 * m * a0.shape[1] * B.shape[1]
        if name in ("conv_nt", "conv_xl"):
            w = args[1]
            ho, wo = _arg(args, kw, 6, "ho"), _arg(args, kw, 7, "wo")
            return 2.0 * a0.shape[0] * ho * wo * w.shape[0] * w.shape[1]
        if name in ("conv_wgrad", "conv_wgrad_xl"):
            x, kh, kwd = args[1], _arg(args, kw, 2, "kh"), _arg(args, kw, 3, "kw")
            return 2.0 * a0.shape[0] * a0.shape[1] * kh * kwd * x.shape[1]
        if name == "conv_xl_dgrad_s2":
            n, _, ho, wo = a0.shape
            return 2.0 * n * ho * wo * sum(w.shape[0] * w.shape[1] for w in args[1])
        if name in ("conv3x3_c64", "conv3x3_c128", "conv3x3_c128_dgrad_s2"):
            w = args[1]
            return 2.0 * _rows4(a0) * w.shape[0] * w.shape[1]
        if name == "wgrad3x3":
            x = args[1]
            return 2.0 * _rows4(a0) * a0.shape[1] * 9 * x.shape[1]
        if name == "stem_halo_fwd":
            wm, ho = args[1], _arg(args, kw, 2, "ho")
            return 2.0 * a0.shape[0] * ho * ho * wm.shape[0] * wm.shape[1]
        if name == "stem_halo_wgrad":
            return 2.0 * _rows4(a0) * 64 * 256
        if name in ("attention_forward", "attention_backward"):
            b, s, h = (args[1], args[2], args[3]) if name == "attention_forward" else (args[4], args[5], args[6])
            f = 4.0 * b * h * s * s * 64
            return f if name == "attention_forward" else 2.5 * f
    except (AttributeError, IndexError, TypeError, ValueError):
        return 0.0
    return 0.0


class _Probe:
    def __init__(self, mod):
        self._mod = mod
        self.records: List[Dict[str, Any]] = []

    def __getattr__(self, name):
        fn = getattr(self._mod, name)
        if not callable(fn) or isinstance(fn, type) or name.startswith(("set_", "get_")) or \
                name.endswith("_supported") or name in ("enable_peer_access", "compute_bucket_assignment"):
            return fn

        def timed(*args, **kw):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = fn(*args, **kw)
            e1.record()
            torch.cuda.synchronize()
            ins = _tensors(args) + _tensors(list(kw.values()))
            shapes = tuple(tuple(t.shape) for t in ins[:3])
            self.records.append({"fn": name, "shapes": shapes, "ms": e0.elapsed_time(e1),
                                 "flops": flops(name, args, kw),
                                 "bytes": _nbytes(ins) + _nbytes(_tensors(out))})
            return out
        return timed


@contextlib.contextmanager
def probe():
    """Route every ``_native.native()`` / ``require()`` lookup through a timing
    proxy for the duration of the block; yields the proxy (``.records``)."""
    from .. import _native
    p = _Probe(_native.require("roofline probe"))
    _native._PROBE = p
    try:
        yield p
    finally:
        _native._PROBE = None


def bound_ms(flops_: float, bytes_: float) -> float:
    return 1e3 * max(flops_ / PEAK_FLOPS, bytes_ / PEAK_BYTES)


def aggregate(records: List[Dict[str, Any]]):
    """Group by (function, leading operand shapes): calls, ms, GFLOP, GB, bound."""
    groups: Dict[tuple, Dict[str, float]] = {}
    for r in records:
        g = groups.setdefault((r["fn"], r["shapes"]), {"calls": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
        g["calls"] += 1
        g["ms"] += r["ms"]
        g["flops"] += r["flops"]
        g["bytes"] += r["bytes"]
    rows = []
    for (fn, shapes), g in groups.items():
        b = bound_ms(g["flops"], g["bytes"])
        kind = "MFMA" if g["flops"] / PEAK_FLOPS > g["bytes"] / PEAK_BYTES else "HBM"
        rows.append(dict(fn=fn, shapes=shapes, calls=g["calls"], ms=g["ms"], gflop=g["flops"] / 1e9,
                         gb=g["bytes"] / 1e9, bound_ms=b, bound=kind,
                         frac=b / g["ms"] if g["ms"] > 0 else 0.0))
    rows.sort(key=lambda r: -r["ms"])
    return rows
