"""Weight gradients on a side HIP stream, concurrent with the data-gradient chain.

In backward, a layer's data gradient dX feeds the next (earlier) layer: that
chain is the step's critical path.  Its weight gradient dW = dY^T X is a leaf
-- only the optimizer (and the DDP bucket all-reduce) read it -- yet eagerly
it sits on the same stream, between two data gradients.  The two kernel kinds
also load the chip differently: one 256 x 256 block per CU in both, so the
partial last round of a data-gradient grid (finding 54: 6.12 rounds cost 7)
leaves CUs idle that a queued weight-gradient grid can fill, and an HBM-bound
BN pass can run beside an MFMA-bound weight gradient.

Mechanism (no change to the autograd graph):
  * every conv / linear backward launches its weight-gradient kernel(s) inside
    :func:`side` -- on a per-device side stream S that first waits for the
    compute stream M (so dY and X are complete), with ``record_stream(S)`` on
    the tensors S reads (the caching allocator must not hand their blocks to
    M's next allocation while S still reads them);
  * the parameters' AccumulateGrad nodes are created ON S (:func:`bind`, and
    DDP builds its reducer under S): autograd then runs AccumulateGrad and its
    post-hooks -- the DDP reducer's bucket flush and all-reduce launch -- on S,
    after the weight-gradient kernels, and at the end of backward the engine
    makes the caller's stream wait for S (its leaf-stream sync), so the
    optimizer on M sees every gradient;
  * a gradient produced on M for a parameter bound to S (BN affine, biases)
    reaches AccumulateGrad through the engine's producer -> consumer event
    (S waits for M: no stall on the critical path).

A parameter whose accumulator is not bound to S (a DataParallel replica, a
model without :func:`bind`) keeps its weight gradient on the compute stream,
and nothing is side-streamed inside a hipGraph capture.  Off by default
(``set_enabled(True)`` turns it on; see ENABLED).
"""
from __future__ import annotations

import contextlib
import weakref
from typing import Dict, Iterable, Iterator, List, Optional

import torch

from .. import _native

# Off by default: measured on MI355X (profiles/README.md finding 57) the side
# stream's kernels only time-slice the CUs with the data-gradient chain at
# batch 2048 (ResNet-50 123.2 ms inline vs 123.8 side; 29 ms of kernels ran
# "concurrently" while the compute queue's own kernels slowed by as much), and
# the per-layer stream handshakes cost launch-bound models host time
# (MobileNetV2 CIFAR 10.9 vs 12.8 ms).  set_enabled(True) enables it.
ENABLED = False


def set_enabled(on: bool) -> None:
    """Weight gradients on the side stream (off by default: finding 56/57).
    Takes effect for models / DDP wrappers built afterwards."""
    global ENABLED
    ENABLED = bool(on) and not _native.disabled("async_wgrad")

_streams: Dict[int, torch.cuda.Stream] = {}
# id(param) -> weakref(param) of parameters whose AccumulateGrad lives on S
_bound: Dict[int, "weakref.ref[torch.Tensor]"] = {}
# strong references to the accumulators created on S (a leaf only weakly
# references its AccumulateGrad: dropped, it would be re-created on M)
_accs: Dict[int, object] = {}
_STATS = {"side": 0, "inline": 0}


def stats() -> dict:
    return dict(_STATS)


def stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        s = _streams[idx] = torch.cuda.Stream(device=idx)
    return s


@contextlib.contextmanager
def creating_on_side(device: torch.device) -> Iterator[None]:
    """Context in which new AccumulateGrad nodes get S as their stream (DDP's
    reducer is built inside it; it holds the accumulators itself)."""
    if not (ENABLED and device.type == "cuda" and torch.cuda.is_available()):
        yield
        return
    if torch.cuda.current_stream(device) != torch.cuda.default_stream(device):
        # the caller manages streams itself (bench --graph builds the whole
        # state on its capture stream, whose accumulators must stay there)
        yield
        return
    s = stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        yield


def _acc_on_side(p: torch.Tensor) -> bool:
    C = _native.native()
    if C is None or not hasattr(C, "grad_accumulator_stream"):
        return False
    return C.grad_accumulator_stream(p) == stream(p.device).stream_id


def mark_bound(params: Iterable[torch.Tensor]) -> int:
    """Bind the leaves whose AccumulateGrad the caller created on S (DDP's
    reducer holds them); a leaf whose accumulator runs on another stream (it
    existed before) stays unbound.  Returns how many were bound."""
    n = 0
    for p in params:
        if ENABLED and p.is_cuda and _acc_on_side(p):
            _bound[id(p)] = weakref.ref(p)
            n += 1
    return n


def bind(params: Iterable[torch.Tensor]) -> List[torch.Tensor]:
    """Create (and keep alive) the AccumulateGrad nodes of ``params`` on the
    side stream.  Leaves that already have an accumulator keep it (it may
    live on M) and are NOT bound.  Returns the bound parameters."""
    out = []
    params = [p for p in params if p.requires_grad and p.is_cuda and p.grad_fn is None]
    if not ENABLED or not params:
        return out
    with creating_on_side(params[0].device):
        for p in params:
            if id(p) in _bound and _bound[id(p)]() is p:
                out.append(p)
                continue
            # p.view_as(p) creates the leaf's accumulator if it has none; if one
            # already exists (created on M) it is reused -- then do not bind
            v = p.view_as(p)
            acc = v.grad_fn.next_functions[0][0]
            if acc is None or not _acc_on_side(p):
                continue
            _accs[id(p)] = acc
            _bound[id(p)] = weakref.ref(p)
            out.append(p)
    return out


def join(device: torch.device) -> None:
    """Make the current stream wait for S (the optimizer does this before its
    update; the engine's end-of-backward leaf-stream sync already should)."""
    if device.type != "cuda":
        return
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is not None and not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream(device).wait_stream(s)


def is_bound(w: torch.Tensor) -> bool:
    r = _bound.get(id(w))
    return r is not None and r() is w


def _active(w: torch.Tensor) -> bool:
    return (ENABLED and w.is_cuda and is_bound(w)
            and not torch.cuda.is_current_stream_capturing())


@contextlib.contextmanager
def side(w: torch.Tensor, *reads: Optional[torch.Tensor]) -> Iterator[None]:
    """Run the enclosed weight-gradient launches for parameter ``w`` on S.

    ``reads``: the tensors the enclosed kernels read that were produced on M
    (dY, X, ...): recorded on S so their memory outlives S's use."""
    if not _active(w):
        _STATS["inline"] += 1
        yield
        return
    _STATS["side"] += 1
    main = torch.cuda.current_stream(w.device)
    s = stream(w.device)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        yield
    for t in reads:
        if t is not None and t.is_cuda:
            t.record_stream(s)
