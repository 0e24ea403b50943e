"""Single-process multi-GPU collectives for DataParallel.

The reference trains with ``nn.DataParallel`` (``data_parallel.py:77``) and
its README walks through the upstream path: scatter (C++), replicate via
``broadcast_coalesced`` in 10 MiB buffers, ``parallel_apply`` threads, gather,
and ``ReduceAddCoalesced`` in backward (Readme.md:17-143).  These are the
MI355X-native equivalents:

* every transfer is a PULL by a kernel on the destination GPU that reads the
  source GPU's memory directly over xGMI (peer access), so the 7 links of the
  8-GPU mesh are driven concurrently by 7 different GPUs instead of one GPU
  pushing serially;
* many tensors move per launch (``_C.multi_copy`` chunk table), no Python loop
  of per-tensor copies, no 10 MiB bucket split (one flat per dtype);
* the reduction of replica gradients is ONE N-way vectorised add kernel on the
  output device reading all peers' flat gradient buffers (``_C.reduce_add_into``);
* gather along dim != 0 uses the LDS-staged tile kernel (``_C.gather_slabs``).

Cross-device ordering is done with HIP events: a consumer stream waits on an
event recorded on the producer's current stream.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from .. import _native
from ..ops import flat as flatops


def _dev(d) -> torch.device:
    if isinstance(d, torch.device):
        return d
    return torch.device("cuda", int(d)) if not isinstance(d, str) else torch.device(d)


# _PEER[a][b]: a kernel on GPU a may dereference GPU b's memory (filled by
# set_peer_matrix from the native enable_peer_access result).  Unknown (None)
# means "never": a peer-pointer kernel over a pair without peer access is a GPU
# fault, a staged copy is merely slower.
_PEER: Optional[List[List[bool]]] = None


def set_peer_matrix(direct: Optional[Sequence[Sequence[bool]]]) -> None:
    global _PEER
    _PEER = [list(map(bool, row)) for row in direct] if direct is not None else None


def peer_ok(reader: torch.device, owner: torch.device) -> bool:
    """May a kernel running on `reader` read `owner`'s memory directly?"""
    reader, owner = _dev(reader), _dev(owner)
    if reader == owner:
        return True
    if reader.type != "cuda" or owner.type != "cuda" or _PEER is None:
        return False
    try:
        return _PEER[reader.index][owner.index]
    except (IndexError, TypeError):
        return False


def _local(ts: Sequence[torch.Tensor], dst: torch.device) -> List[torch.Tensor]:
    """`ts` made readable by a kernel on `dst`: tensors on a device `dst` has no
    peer mapping to are first copied over by the runtime (staged
    hipMemcpyPeerAsync behind torch's copy_, ordered on both current streams)."""
    return [t if peer_ok(dst, t.device) else t.to(dst, non_blocking=True) for t in ts]


def _wait_for(src_dev: torch.device, dst_dev: torch.device) -> None:
    """Make dst's current stream wait for work already queued on src's current stream."""
    if src_dev.type != "cuda" or dst_dev.type != "cuda" or src_dev == dst_dev:
        return
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(src_dev))
    torch.cuda.current_stream(dst_dev).wait_event(ev)


def _keep_alive(srcs: Sequence[torch.Tensor], consumer: torch.device) -> None:
    """A kernel on `consumer` reads these peer tensors: tell each source device's
    caching allocator not to reuse the memory before the consumer stream is done
    (the Python references may die as soon as the launch returns)."""
    if consumer.type != "cuda":
        return
    stream = torch.cuda.current_stream(consumer)
    for t in srcs:
        if t.is_cuda and t.device != consumer:
            t.record_stream(stream)


def pull_copy(srcs: Sequence[torch.Tensor], dsts: Sequence[torch.Tensor]) -> None:
    """dst[i] <- src[i]; one kernel on dst's device reading (possibly peer) sources."""
    if not srcs:
        return
    dd = dsts[0].device
    if dd.type == "cuda" and not all(peer_ok(dd, t.device) for t in srcs):
        direct = [(a, b) for a, b in zip(srcs, dsts) if peer_ok(dd, a.device)]
        with torch.no_grad():
            for a, b in zip(srcs, dsts):
                if not peer_ok(dd, a.device):
                    b.copy_(a, non_blocking=True)  # staged: no peer mapping for this pair
        if direct:
            pull_copy([a for a, _ in direct], [b for _, b in direct])
        return
    for s in {t.device for t in srcs}:
        _wait_for(s, dd)
    _keep_alive(srcs, dd)
    if dd.type == "cuda":
        with torch.cuda.device(dd):
            _native.require("DataParallel pull copy").multi_copy(list(srcs), list(dsts))
    else:
        with torch.no_grad():
            for s, d in zip(srcs, dsts):
                d.copy_(s)


# --------------------------------------------------------------------------- #
# broadcast / reduce_add (coalesced)
# --------------------------------------------------------------------------- #
def broadcast_coalesced(tensors: Sequence[torch.Tensor], devices: Sequence,
                        ) -> List[List[torch.Tensor]]:
    """Copy `tensors` (all on devices[0]) to every device; returns per-device lists.

    devices[0]'s entry aliases the inputs (like upstream).  One flatten launch on
    the source, then each destination pulls the flat buffer and unflattens with
    one launch each.
    """
    devices = [_dev(d) for d in devices]
    out: List[List[torch.Tensor]] = [list(tensors)]
    if len(devices) == 1 or not tensors:
        return out + [[] for _ in devices[1:]]
    groups = flatops.group_by_dtype(tensors)
    flats = {k: flatops.flatten([tensors[i] for i in idxs]) for k, idxs in groups.items()}
    for d in devices[1:]:
        res: List[Optional[torch.Tensor]] = [None] * len(tensors)
        for k, idxs in groups.items():
            src_flat = flats[k]
            dst_flat = torch.empty(src_flat.numel(), dtype=src_flat.dtype, device=d)
            pull_copy([src_flat], [dst_flat])
            offs, _ = flatops.flat_layout([tensors[i] for i in idxs])
            with torch.cuda.device(d) if d.type == "cuda" else _null():
                for i, o in zip(idxs, offs):
                    t = tensors[i]
                    v = dst_flat.narrow(0, o, t.numel())
                    res[i] = _shape_like(v, t)
        out.append(res)  # type: ignore[arg-type]
    return out


def _shape_like(flat_slice: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
    """View a flat slice with `like`'s shape and memory format (memory order)."""
    if like.is_contiguous():
        return flat_slice.view(like.shape)
    if like.dim() == 4 and like.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = like.shape
        return flat_slice.view(n, h, w, c).permute(0, 3, 1, 2)
    return flat_slice.view(like.shape)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def reduce_add_coalesced(grads_per_device: Sequence[Sequence[torch.Tensor]],
                         destination) -> List[torch.Tensor]:
    """Sum per-device tensor lists onto `destination` (one N-way add kernel per dtype)."""
    dst = _dev(destination)
    n = len(grads_per_device[0])
    out: List[Optional[torch.Tensor]] = [None] * n
    ref = grads_per_device[0]
    groups = flatops.group_by_dtype([t if t is not None else torch.empty(0) for t in ref])
    for (_dt, _d), idxs in groups.items():
        like = [ref[i] for i in idxs]
        flats = []
        for dev_list in grads_per_device:
            ts = [dev_list[i] for i in idxs]
            flats.append(flatops.flatten(ts))
        total = flats[0].numel()
        res = torch.empty(total, dtype=flats[0].dtype, device=dst)
        if dst.type == "cuda":
            flats = _local(flats, dst)
        for f in flats:
            _wait_for(f.device, dst)
        _keep_alive(flats, dst)
        if dst.type == "cuda":
            with torch.cuda.device(dst):
                _native.require("reduce_add").reduce_add_into(flats, res)
        else:
            res.copy_(torch.stack([f.to(dst) for f in flats]).sum(0))
        offs, _ = flatops.flat_layout(like)
        for i, o, t in zip(idxs, offs, like):
            out[i] = _shape_like(res.narrow(0, o, t.numel()), t)
    return out  # type: ignore[return-value]


# --------------------------------------------------------------------------- #
# scatter / gather
# --------------------------------------------------------------------------- #
def _chunk_sizes(n: int, parts: int) -> List[int]:
    base = (n + parts - 1) // parts
    sizes = []
    left = n
    while left > 0 and len(sizes) < parts:
        s = min(base, left)
        sizes.append(s)
        left -= s
    return sizes


def scatter_tensor(t: torch.Tensor, devices: Sequence, dim: int = 0,
                   chunk_sizes: Optional[Sequence[int]] = None) -> List[torch.Tensor]:
    devices = [_dev(d) for d in devices]
    sizes = list(chunk_sizes) if chunk_sizes is not None else _chunk_sizes(t.shape[dim], len(devices))
    chunks = torch.split(t, sizes, dim)
    outs = []
    for c, d in zip(chunks, devices):
        if c.device == d:
            outs.append(c)
            continue
        dst = torch.empty(c.shape, dtype=c.dtype, device=d,
                          memory_format=torch.channels_last
                          if (c.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last)
                              and not t.is_contiguous()) else torch.contiguous_format)
        if d.type == "cuda" and c.is_cuda:
            src = c if (c.is_contiguous() or c.is_contiguous(memory_format=torch.channels_last)) \
                else c.contiguous()
            sraw = flatops.raw_view(src)
            draw = flatops.raw_view(dst)
            if sraw is not None and draw is not None and src.stride() == dst.stride():
                pull_copy([sraw], [draw])
            else:
                _wait_for(c.device, d)
                dst.copy_(c)
        else:
            dst.copy_(c)
        outs.append(dst)
    return outs


def gather_tensors(ts: Sequence[torch.Tensor], destination, dim: int = 0) -> torch.Tensor:
    dst = _dev(destination)
    ts = [t if t.dim() > 0 else t.view(1) for t in ts]
    shape = list(ts[0].shape)
    shape[dim] = sum(t.shape[dim] for t in ts)
    out = torch.empty(shape, dtype=ts[0].dtype, device=dst)
    if dst.type != "cuda":
        return torch.cat([t.to(dst) for t in ts], dim, out=out)
    ts = _local(ts, dst)
    for t in ts:
        _wait_for(t.device, dst)
    srcs = [t.contiguous() for t in ts]
    _keep_alive(srcs, dst)
    if dim == 0:
        views = [s.view(s.shape[0], -1) for s in srcs]
        out2 = out.view(shape[0], -1)
    else:
        lead = 1
        for s in shape[:dim]:
            lead *= s
        views = [s.view(lead, -1) for s in srcs]
        out2 = out.view(lead, -1)
    with torch.cuda.device(dst):
        _native.require("gather").gather_slabs(views, out2, dim != 0)
    return out
