"""Flatten / unflatten many tensors with one HIP launch (``_C.multi_copy``).

Used for coalesced broadcasts (DDP module-state sync, DataParallel replicate)
and for packing gradients.  CPU tensors use ``torch.cat``-style copies.
Buffers produced here pad each tensor to 16 bytes so every slice stays
16-byte aligned for the vectorised kernels.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch

from .. import _native


def _pad_elems(t: torch.Tensor) -> int:
    per = max(1, 16 // t.element_size())
    return (t.numel() + per - 1) // per * per


def flat_layout(tensors: Sequence[torch.Tensor]) -> Tuple[List[int], int]:
    offs, o = [], 0
    for t in tensors:
        offs.append(o)
        o += _pad_elems(t)
    return offs, o


def raw_view(t: torch.Tensor):
    """1-D view of a dense tensor's memory (contiguous or channels-last), else None."""
    if t.is_contiguous():
        return t.view(-1)
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).reshape(-1)
    return None


def multi_copy_(srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor]) -> None:
    """dst[i].copy_(src[i]) for all i; one launch on GPU (sources may be on peers)."""
    if not srcs:
        return
    if dsts[0].is_cuda:
        _native.require("multi_copy").multi_copy([s.contiguous() for s in srcs], list(dsts))
    else:
        with torch.no_grad():
            for s, d in zip(srcs, dsts):
                d.copy_(s)


def flatten(tensors: Sequence[torch.Tensor], out: torch.Tensor = None) -> torch.Tensor:
    """Pack same-dtype tensors into one flat buffer (16-B aligned slices)."""
    assert tensors, "flatten needs at least one tensor"
    offs, total = flat_layout(tensors)
    if out is None:
        out = torch.zeros(total, dtype=tensors[0].dtype, device=tensors[0].device)
    views = [out.narrow(0, o, t.numel()) for o, t in zip(offs, tensors)]
    srcs = []
    for t in tensors:
        r = raw_view(t)
        srcs.append(r if r is not None else t.contiguous().view(-1))
    multi_copy_(srcs, views)
    return out


def unflatten_into(flat: torch.Tensor, tensors: Sequence[torch.Tensor]) -> None:
    """Copy slices of `flat` (layout from :func:`flat_layout`) back into `tensors`."""
    offs, _ = flat_layout(tensors)
    raws = [raw_view(t) for t in tensors]
    if all(r is not None for r in raws):
        multi_copy_([flat.narrow(0, o, t.numel()) for o, t in zip(offs, tensors)], raws)
    else:
        with torch.no_grad():
            for o, t, r in zip(offs, tensors, raws):
                src = flat.narrow(0, o, t.numel())
                if r is not None:
                    r.copy_(src)
                else:
                    t.copy_(src.view(t.shape))


def group_by_dtype(tensors: Sequence[torch.Tensor]):
    groups = {}
    for i, t in enumerate(tensors):
        groups.setdefault((t.dtype, t.device), []).append(i)
    return groups
