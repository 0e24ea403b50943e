"""Checkpoint / resume.

Reference behaviour (``data_parallel.py:80-87,143-155``): save
``{'net': state_dict, 'acc', 'epoch'}`` to ``./checkpoint/ckpt.pth`` when val
accuracy improves, resume with ``-r``; keys carry the DataParallel
``module.`` prefix; no optimizer/scheduler/RNG state; the pipeline script
saves nothing.

Here: rank-0 atomic save (temp file + rename) of the model state
(``module.``-prefixed when the model is wrapped, as in the reference; loading
accepts either) with ``weights_only=True``-safe contents, optimizer, scheduler,
epoch, best accuracy and RNG states; per-stage shards for pipeline runs;
``load_checkpoint`` maps onto the local device and (under DDP) re-broadcasts
from rank 0 so every replica resumes bit-identical.
"""
from __future__ import annotations

import os
import pickle
import random
import warnings
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
    """RNG states as tensors / ints / tuples only, so the file loads with
    ``torch.load(weights_only=True)`` (no pickled numpy objects)."""
    name, keys, pos, has_gauss, gauss = np.random.get_state()
    st = {"python": random.getstate(),
          "numpy": [name, torch.from_numpy(np.asarray(keys, dtype=np.int64)), int(pos),
                    int(has_gauss), float(gauss)],
          "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st: Dict[str, Any]) -> None:
    random.setstate(st["python"])
    name, keys, pos, has_gauss, gauss = st["numpy"]
    # current format: keys as an int64 tensor; legacy files: np.random.get_state()'s ndarray
    keys = keys.numpy() if isinstance(keys, torch.Tensor) else np.asarray(keys)
    np.random.set_state((name, keys.astype(np.uint32), int(pos), int(has_gauss), float(gauss)))
    torch.set_rng_state(st["torch"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["cuda"])


def _rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def save_checkpoint(path: str, model: nn.Module, optimizer=None, scheduler=None, epoch: int = 0,
                    best_acc: float = 0.0, extra: Optional[Dict[str, Any]] = None,
                    all_ranks: bool = False, module_prefix: Optional[bool] = None) -> Optional[str]:
    """Write a checkpoint (rank 0 only unless `all_ranks`, e.g. pipeline shards).

    ``module_prefix`` (default: whether `model` is a DP/DDP wrapper) writes the
    ``net`` keys with the ``module.`` prefix the reference's DataParallel
    checkpoints carry (``data_parallel.py:143-155``), so its
    ``net.load_state_dict(checkpoint['net'])`` accepts our files too.
    """
    if not all_ranks and _rank() != 0:
        return None
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    net = unwrap(model).state_dict()
    if module_prefix is None:
        module_prefix = unwrap(model) is not model
    if module_prefix:
        net = {"module." + k: v for k, v in net.items()}
    state = {
        "net": net,
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
    state = _load_weights_only(path, map_location)
    target = unwrap(model)
    target.load_state_dict(_strip_prefix(state["net"]), strict=strict)
    restored = False
    if optimizer is not None and state.get("optimizer") is not None:
        from ..ops.optim import ForeignOptimizerState
        sd = state["optimizer"]
        ours = hasattr(optimizer, "sync_from_params")  # FlatSGD / MasterSGD
        if ours:
            try:
                optimizer.load_state_dict(sd)
                restored = True
            except ForeignOptimizerState as e:  # e.g. a torch.optim.SGD state from an older DP run
                warnings.warn(f"load_checkpoint: optimizer state not restored ({e}); starting it "
                              "fresh from the loaded weights")
            # any other error (a layout that differs from the checkpoint) propagates
        else:
            optimizer.load_state_dict(sd)
            restored = True
    if optimizer is not None and not restored and hasattr(optimizer, "sync_from_params"):
        # weights came without (usable) optimizer state: the fp32 masters must follow them
        optimizer.sync_from_params()
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


def _load_weights_only(path: str, map_location):
    """``torch.load(weights_only=True)``: tensors / containers / numbers only,
    nothing in the file is executed.  Files written before the RNG state became
    tensor-only pickle ``np.random.get_state()``'s uint32 ndarray; for those the
    numpy array *reconstructors* (plain data constructors, no code) are
    allow-listed and the load retried, still weights-only."""
    try:
        return torch.load(path, map_location=map_location, weights_only=True)
    except pickle.UnpicklingError:
        allowed = [np.ndarray, np.dtype]
        try:
            from numpy.core.multiarray import _reconstruct  # numpy >= 2 keeps this alias
            allowed.append(_reconstruct)
        except ImportError:  # pragma: no cover
            pass
        allowed.extend(t for t in (getattr(np, "dtypes", None) and getattr(np.dtypes, "UInt32DType", None),)
                       if t is not None)
        with torch.serialization.safe_globals(allowed):
            return torch.load(path, map_location=map_location, weights_only=True)


def stage_checkpoint_path(path: str, stage: int) -> str:
    root, ext = os.path.splitext(path)
    return f"{root}.stage{stage}{ext or '.pth'}"
