"""Spawn a local gloo world (127.0.0.1) and collect per-rank results."""
from __future__ import annotations

import os
import socket
import tempfile
import traceback

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    ok = False
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        torch.save({"ok": True, "res": res}, os.path.join(outdir, f"r{rank}.pt"))
        ok = True
    except Exception:  # noqa: BLE001
        torch.save({"ok": False, "err": traceback.format_exc()}, os.path.join(outdir, f"r{rank}.pt"))
        raise
    finally:
        if dist.is_initialized():
            from distributed_model_parallel_amd.comm.rccl import reset_default_communicator
            from distributed_model_parallel_amd.utils.env import destroy_distributed
            reset_default_communicator()
            if ok:
                # barrier + rank-0 store linger (a peer tearing down against a dead
                # store aborted with "terminate called without an active exception")
                destroy_distributed()
            else:  # a failed rank: its peers may never reach a barrier
                dist.destroy_process_group()


def run_world(fn, world: int, *args):
    """Run fn(rank, world, *args) in `world` gloo processes; return list of results."""
    with tempfile.TemporaryDirectory() as d:
        port = free_port()
        try:
            mp.spawn(_entry, args=(world, port, fn, args, d), nprocs=world, join=True)
        except Exception:
            errs = []
            for r in range(world):
                p = os.path.join(d, f"r{r}.pt")
                if os.path.exists(p):
                    o = torch.load(p, weights_only=False)
                    if not o["ok"]:
                        errs.append(f"rank {r}:\n{o['err']}")
            raise AssertionError("\n".join(errs) or "worker failed")
        out = []
        for r in range(world):
            o = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=False)
            out.append(o["res"])
        return out


def run_world_exitcodes(fn, world: int, *args, timeout_s: float = 60.0):
    """Run fn(rank, world, *args) in `world` gloo processes without joining on
    success; returns each process's exit code (None = still running when the
    timeout expired; such processes are then killed)."""
    import time
    port = free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_exit_entry, args=(r, world, port, fn, args), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    deadline = time.monotonic() + timeout_s
    for p in procs:
        p.join(max(0.0, deadline - time.monotonic()))
    codes = [p.exitcode for p in procs]
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join(5)
    return codes


def _exit_entry(rank, world, port, fn, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fn(rank, world, *args)
