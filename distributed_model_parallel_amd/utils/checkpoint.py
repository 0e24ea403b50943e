"""Checkpoint / resume.

Reference behaviour (``data_parallel.py:80-87,143-155``): save
``{'net': state_dict, 'acc', 'epoch'}`` to ``./checkpoint/ckpt.pth`` when val
accuracy improves, resume with ``-r``; keys carry the DataParallel
``module.`` prefix; no optimizer/scheduler/RNG state; the pipeline script
saves nothing.

Here: rank-0 atomic save (temp file + rename) of the UNWRAPPED model state
(no ``module.`` prefix; loading accepts either), optimizer, scheduler,
epoch, best accuracy and RNG states; per-stage shards for pipeline runs;
``load_checkpoint`` maps onto the local device and (under DDP) re-broadcasts
from rank 0 so every replica resumes bit-identical.
"""
from __future__ import annotations

import os
import random
from typing import Any, Dict, Optional

import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn


def unwrap(model: nn.Module) -> nn.Module:
    while hasattr(model, "module") and isinstance(model.module, nn.Module):
        model = model.module
    return model


def _strip_prefix(sd: Dict[str, Any], prefix: str = "module.") -> Dict[str, Any]:
    if sd and all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return sd


def rng_state() -> Dict[str, Any]:
    st = {"python": random.getstate(), "numpy": np.random.get_state(), "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st: Dict[str, Any]) -> None:
    random.setstate(st["python"])
    np.random.set_state(st["numpy"])
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["cuda"])


def _rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def save_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None, epoch: int = 0,
                    best_acc: float = 0.0, extra: Optional[Dict[str, Any]] = None,
                    all_ranks: bool = False) -> Optional[str]:
    """Write a checkpoint (rank 0 only unless `all_ranks`, e.g. pipeline shards)."""
    if not all_ranks and _rank() != 0:
        return None
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    state = {
        "net": unwrap(model).state_dict(),
        "acc": best_acc,
        "epoch": epoch,
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "scheduler": scheduler.state_dict() if scheduler is not None and hasattr(scheduler, "state_dict") else None,
        "rng": rng_state(),
        "extra": extra or {},
    }
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(state, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None,
                    map_location=None, restore_rng: bool = True, strict: bool = True) -> Dict[str, Any]:
    """Load a checkpoint written by :func:`save_checkpoint` (or the reference's
    ``{'net','acc','epoch'}`` dict) into `model` / `optimizer` / `scheduler`."""
    if map_location is None:
        map_location = "cpu"
    # our own files; weights_only=False is needed for RNG/optimizer state objects
    state = torch.load(path, map_location=map_location, weights_only=False)
    target = unwrap(model)
    target.load_state_dict(_strip_prefix(state["net"]), strict=strict)
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler") is not None:
        scheduler.load_state_dict(state["scheduler"])
    if restore_rng and state.get("rng") is not None:
        try:
            set_rng_state(state["rng"])
        except Exception:  # noqa: BLE001 - RNG layout differs across device counts
            pass
    ddp = model if hasattr(model, "reducer") else None
    if ddp is not None and ddp.world_size > 1:
        ddp._sync_module_states()
    return {"epoch": state.get("epoch", 0), "acc": state.get("acc", 0.0), "extra": state.get("extra", {})}


def stage_checkpoint_path(path: str, stage: int) -> str:
    root, ext = os.path.splitext(path)
    return f"{root}.stage{stage}{ext or '.pth'}"
