"""Process bootstrap: one process per GPU, torchrun environment.

Reference parity: ``model_parallel.py:52-61,162`` spawns one process per GPU
with ``mp.spawn`` and a hard-coded ``tcp://127.0.0.1:1224`` rendezvous.  Here
the canonical launcher is ``torchrun`` (``env://``: RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT), with an ``mp.spawn``-style helper for
tests and the reference's ``--dist-url`` still accepted.

On GPU the torch process group uses the ``nccl`` backend (= RCCL on ROCm) and
is only used as a rendezvous store / control plane; bulk data moves through
the native :class:`~..comm.rccl.Communicator`.  On CPU it is ``gloo``.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    device: torch.device = torch.device("cpu")

    @property
    def is_main(self) -> bool:
        return self.rank == 0

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


def env_int(name: str, default: int) -> int:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def single_rank_comm() -> bool:
    """Run the collectives even at world size 1 (measurement mode: the DDP
    bucket all-reduces and the SyncBN moment all-reduces then really go through
    RCCL instead of being skipped as identities).  ``DMP_SINGLE_RANK_COMM=1``;
    the round-2 name ``DMP_DDP_SINGLE_RANK_COMM=1`` is still honoured."""
    return os.environ.get("DMP_SINGLE_RANK_COMM", os.environ.get("DMP_DDP_SINGLE_RANK_COMM", "0")) == "1"


def count_gpus_without_hip() -> Optional[int]:
    """Number of visible GPUs, read WITHOUT initialising the HIP runtime (for
    launcher processes that must stay GPU-free): the *_VISIBLE_DEVICES lists
    when set, else the KFD topology nodes that have SIMDs.  None = unknown
    (let the ranks validate)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        n = 0
        for node in os.listdir(root):
            with open(os.path.join(root, node, "properties")) as f:
                for line in f:
                    k, _, val = line.partition(" ")
                    if k == "simd_count" and int(val) > 0:
                        n += 1
                        break
        return n
    except (OSError, ValueError):
        return None


def read_env() -> DistEnv:
    rank = env_int("RANK", 0)
    ws = env_int("WORLD_SIZE", 1)
    lr = env_int("LOCAL_RANK", rank)
    lws = env_int("LOCAL_WORLD_SIZE", ws)
    return DistEnv(rank, ws, lr, lws)


def init_distributed(backend: Optional[str] = None, dist_url: Optional[str] = None,
                     timeout_s: float = 1800.0, use_gpu: Optional[bool] = None) -> DistEnv:
    """Initialise torch.distributed from the torchrun environment (idempotent).

    Sets the current device to LOCAL_RANK when GPUs are present.  Always
    creates a process group (also for world_size 1) so the same code path runs
    at every scale.
    """
    e = read_env()
    if use_gpu is None:
        use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(e.local_rank)
        e.device = torch.device("cuda", e.local_rank)
    if backend is None:
        backend = "nccl" if use_gpu else "gloo"
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=e.rank, world_size=e.world_size,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if e.world_size == 1 and dist_url is None:
            # one rank: an in-process store, no TCP rendezvous -- a port picked
            # for it can be taken by another process between the pick and the
            # bind (EADDRINUSE on shared boxes)
            kw["store"] = dist.HashStore()
        else:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + (os.getpid() % 1000)))
            kw["init_method"] = dist_url or "env://"
        dist.init_process_group(**kw)
    return e


def destroy_distributed() -> None:
    if dist.is_initialized():
        linger = False
        if dist.get_backend() == "gloo" and dist.get_world_size() > 1:
            # every rank reaches the teardown before any closes its pairs: a gloo
            # process group destroyed while a peer still drains the last
            # collective aborted that peer ("terminate called without an active
            # exception", ~1 in 4 four-rank CPU pipeline benches).  Bounded: a
            # peer that failed never arrives, and then we tear down anyway.
            try:
                import datetime
                dist.monitored_barrier(timeout=datetime.timedelta(seconds=60))
            except RuntimeError:
                pass
            # and rank 0 hosts the TCP store: if it exits first, a peer still
            # tearing down polls a dead store ("... could not be retrieved.
            # err=-3") and aborts the same way (seen once in a round-6 CPU suite)
            linger = dist.get_rank() == 0
        dist.destroy_process_group()
        if linger:
            import time
            time.sleep(1.0)


def seed_everything(seed: int) -> None:
    import random

    import numpy as np

    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)
