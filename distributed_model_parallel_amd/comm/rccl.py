"""Native RCCL communicator (``_C.RcclComm``) bootstrapped through the
torch.distributed store.

Why our own communicator instead of the process group's collectives: the DDP
reducer issues all-reduces from C++ autograd hooks on a dedicated
dedicated HIP stream and never touches Python or the c10d work objects in
the backward path; pipeline P2P uses the same communicator with a static
shape contract (no host round-trips).

``Communicator`` also provides CPU (gloo) equivalents of every call so the
same Python code runs in CPU tests.
"""
from __future__ import annotations

import itertools
import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .. import _native

_counter = itertools.count()

# Every communicator this process created, in creation order, with what decides
# its stream's hardware queue: (purpose, group ranks, device type, priority,
# inline).  DDP's bucket communicator and SyncBatchNorm's moment communicator
# drive two streams; with GPU_MAX_HW_QUEUES (4) those streams may share a
# hardware queue, where kernels execute in submission order.  A cross-
# communicator deadlock needs two ranks whose queues hold the two collectives
# in opposite orders.  The merged submission order is rank-independent
# (parallel/sync_batchnorm.py, "Ordering"); the stream -> queue assignment is
# the runtime's round-robin over streams in creation order, so it is the same
# on every rank exactly when the communicators (and their streams) were
# created in the same order with the same flags -- which verify_comm_layout()
# asserts instead of assuming.
_LAYOUT: list = []


def _store():
    return dist.distributed_c10d._get_default_store()


class Communicator:
    """Collectives + P2P over RCCL (GPU) or the default process group (CPU).

    All GPU operations are asynchronous on the communicator's own stream,
    ordered after the caller's current stream; call :meth:`wait` to make the
    current stream depend on them, or :meth:`synchronize` to block the host.
    """

    def __init__(self, device: torch.device, group: Optional[dist.ProcessGroup] = None,
                 purpose: str = "generic"):
        self.device = torch.device(device)
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        self.purpose = purpose
        self._comm = None
        ranks = None if group is None else tuple(dist.get_process_group_ranks(group))
        _LAYOUT.append((purpose, ranks, self.device.type, os.environ.get("DMP_COMM_INLINE", "0")))
        if self.device.type == "cuda":
            C = _native.require("RCCL communicator")
            key = f"dmp/rccl_uid/{next(_counter)}"
            store = _store()
            if self.rank == 0:
                uid = C.RcclComm.new_unique_id()
                store.set(key, uid)
            else:
                uid = store.get(key)
            # NOT high priority: a high-priority HIP stream slowed the whole ResNet-50
            # step 1.9x on MI355X (67.3 vs 36.5 ms, profiles/README.md finding 1)
            self._comm = C.RcclComm(bytes(uid), self.size, self.rank, self.device.index, False)
            # DMP_COMM_INLINE=1: collectives on the compute stream (no overlap, no side queue)
            if os.environ.get("DMP_COMM_INLINE", "0") == "1":
                self._comm.set_inline(True)

    # ------------------------------------------------------------------ #
    @property
    def native(self):
        """The underlying ``_C.RcclComm`` (None on CPU)."""
        return self._comm

    def all_reduce(self, t: torch.Tensor, op: str = "sum", on_current_stream: bool = False) -> torch.Tensor:
        """In place.  Default: on the communicator's side stream (call wait()
        before consuming).  on_current_stream: enqueued on the caller's stream
        (for small collectives needed immediately; no wait() required)."""
        if self._comm is not None:
            self._comm.all_reduce(t, op, on_current_stream)
            return t
        if op == "avg":
            dist.all_reduce(t, group=self.group)
            t.div_(self.size)
        else:
            dist.all_reduce(t, op=_torch_op(op), group=self.group)
        return t

    def all_reduce_coalesced(self, ts: Sequence[torch.Tensor], op: str = "sum") -> None:
        if self._comm is not None:
            self._comm.all_reduce_coalesced(list(ts), op)
            return
        for t in ts:
            self.all_reduce(t, op)

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        if self._comm is not None:
            self._comm.broadcast(t, root)
        else:
            dist.broadcast(t, src=dist.get_global_rank(self.group, root) if self.group else root,
                           group=self.group)
        return t

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        if self._comm is not None:
            self._comm.all_gather(out, inp)
        else:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        return out

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self._comm is not None:
            self._comm.reduce_scatter(out, inp, op)
        else:
            chunks = list(inp.chunk(self.size))
            tmp = [c.clone() for c in chunks]
            for t in tmp:
                dist.all_reduce(t, group=self.group)
            out.copy_(tmp[self.rank] / (self.size if op == "avg" else 1))
        return out

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        if self._comm is not None:
            self._comm.all_to_all(out, inp)
        else:
            dist.all_to_all_single(out, inp, group=self.group)
        return out

    def send(self, t: torch.Tensor, peer: int) -> None:
        if self._comm is not None:
            self._comm.send(t, peer)
        else:
            dist.send(t, dst=peer, group=self.group)

    def recv(self, t: torch.Tensor, peer: int) -> torch.Tensor:
        if self._comm is not None:
            self._comm.recv(t, peer)
        else:
            dist.recv(t, src=peer, group=self.group)
        return t

    def batch_p2p(self, ops: List[tuple]) -> None:
        """ops: list of (tensor, peer, is_send); issued as one RCCL group."""
        if not ops:
            return
        if self._comm is not None:
            self._comm.batch_p2p([o[0] for o in ops], [int(o[1]) for o in ops], [bool(o[2]) for o in ops])
            return
        reqs = [dist.P2POp(dist.isend if s else dist.irecv, t, p, group=self.group) for t, p, s in ops]
        for r in dist.batch_isend_irecv(reqs):
            r.wait()

    def wait(self) -> None:
        if self._comm is not None:
            self._comm.wait()

    def synchronize(self) -> None:
        if self._comm is not None:
            self._comm.synchronize()

    def barrier(self) -> None:
        """Device+host barrier: tiny all-reduce, then block until done."""
        if self._comm is not None:
            t = torch.zeros(1, device=self.device)
            self._comm.all_reduce(t, "sum")
            self._comm.synchronize()
        else:
            dist.barrier(group=self.group)

    def max_scalar(self, v: float) -> float:
        t = torch.tensor([float(v)], dtype=torch.float64,
                         device=self.device if self._comm is not None else "cpu")
        self.all_reduce(t, "max")
        self.synchronize()
        return float(t.item())


def _torch_op(op: str):
    return {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN,
            "prod": dist.ReduceOp.PRODUCT}[op]


_default: Optional[Communicator] = None


def comm_layout() -> list:
    """This process's communicators in creation order (see _LAYOUT)."""
    return list(_LAYOUT)


def verify_comm_layout(where: str = "", group: Optional[dist.ProcessGroup] = None) -> int:
    """Collective over ``group``: raise on every rank unless all its ranks
    created the same communicators in the same order with the same stream
    flags.  Returns the layout digest."""
    import zlib
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return 0
    dig = zlib.crc32(repr(_LAYOUT).encode())
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([dig, -dig], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    if int(t[0]) != dig or int(t[1]) != -dig:
        raise RuntimeError(f"communicator layout differs across ranks{' at ' + where if where else ''}: this "
                           f"rank created {_LAYOUT}; collectives of different communicators could then share "
                           "hardware queues in different orders on different ranks and deadlock")
    return dig


def default_communicator(device: Optional[torch.device] = None) -> Communicator:
    """Process-wide communicator over the default group (created lazily)."""
    global _default
    if _default is None:
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
                else torch.device("cpu")
        _default = Communicator(device, purpose="default")
    return _default


def reset_default_communicator() -> None:
    """Forget the process-wide communicators (default + SyncBN's own)."""
    global _default
    _default = None
    _LAYOUT.clear()
    from ..parallel.sync_batchnorm import reset_syncbn_communicators
    reset_syncbn_communicators()
