"""Tracing ranges and profiler helpers.

``trace_range(name)`` emits an roctx range (visible in ``rocprofv3
--marker-trace`` / ``--sys-trace`` timelines) around scatter / replicate /
apply / gather, each DDP bucket, pipeline hops, etc.  roctx is called through
ctypes on the ``libroctx64`` PyTorch already ships, so there is no build-time
dependency; when the library is missing the ranges are no-ops.
``torch_profile`` wraps ``torch.profiler`` for a quick operator table.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Iterator, Optional

_roctx = None
_tried = False


def _lib():
    global _roctx, _tried
    if _tried:
        return _roctx
    _tried = True
    if os.environ.get("DMP_DISABLE_ROCTX") == "1":
        return None
    # rocprofiler-sdk's roctx first -- what rocprofv3 --marker-trace intercepts (the
    # native reducer resolves the same library, csrc/trace.h) -- then the legacy
    # roctracer one (torch's bundled copy last: rocprofv3 does not see it)
    cands = ["librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
             "libroctx64.so", "/opt/rocm/lib/libroctx64.so"]
    try:
        import torch
        cands.append(os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"))
    except Exception:  # noqa: BLE001
        pass
    for c in cands:
        if os.path.isabs(c) and not os.path.exists(c):
            continue
        try:
            lib = ctypes.CDLL(c, mode=ctypes.RTLD_GLOBAL)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            break
        except (OSError, AttributeError):
            continue
    return _roctx


def available() -> bool:
    return _lib() is not None


def mark(msg: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(msg.encode())


def push(name: str) -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop() -> None:
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


@contextlib.contextmanager
def trace_range(name: str) -> Iterator[None]:
    lib = _lib()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


@contextlib.contextmanager
def torch_profile(path: Optional[str] = None, cuda: bool = True, row_limit: int = 30):
    """Profile the enclosed region with torch.profiler; print a table and
    optionally export a chrome trace to `path`."""
    import torch
    acts = [torch.profiler.ProfilerActivity.CPU]
    if cuda and torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    key = "self_cuda_time_total" if len(acts) > 1 else "self_cpu_time_total"
    print(prof.key_averages().table(sort_by=key, row_limit=row_limit))
    if path:
        prof.export_chrome_trace(path)


# --------------------------------------------------------------------------- #
# Per-phase GPU time (bench.py --phase-times): HIP events recorded on the
# current stream around each named phase, summed per name.  Off by default
# (no events, no syncs); the roctx range is emitted either way.
_PHASES = None  # name -> list of (start_event, end_event)


def enable_phase_timing(on: bool = True) -> None:
    global _PHASES
    _PHASES = {} if on else None


@contextlib.contextmanager
def phase(name: str) -> Iterator[None]:
    """roctx range + (when enabled) a start/end HIP event pair on the current stream."""
    if _PHASES is None:
        with trace_range(name):
            yield
        return
    import torch
    if not torch.cuda.is_available():
        with trace_range(name):
            yield
        return
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    with trace_range(name):
        a.record()
        try:
            yield
        finally:
            b.record()
    _PHASES.setdefault(name, []).append((a, b))


def phase_summary(reset: bool = True) -> dict:
    """{name: {"ms": total GPU ms, "calls": n}} over everything since the last reset
    (synchronises the device)."""
    global _PHASES
    if not _PHASES:
        return {}
    import torch
    torch.cuda.synchronize()
    out = {k: {"ms": round(sum(a.elapsed_time(b) for a, b in v), 3), "calls": len(v)}
           for k, v in _PHASES.items()}
    if reset:
        _PHASES = {}
    return out
