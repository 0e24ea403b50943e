"""Offline-tuned hipBLASLt / rocBLAS solutions for the library GEMMs.

The transformer linears (ViT qkv / proj / fc1 / fc2 in their forward, data-
and weight-gradient forms) stay on the vendor GEMM libraries: on those short-K
shapes they are as fast as our own MFMA kernels (tools/vit_bench.py --xl,
profiles/vit_gemm_backends.md).  What the libraries do NOT do is pick the best
of their own solutions: the default heuristic leaves 10-30 % on the table for
the [25216 x 768]-type operands of ViT-B/16 at batch 128.  PyTorch's TunableOp
times every hipBLASLt and rocBLAS solution for a shape once; the winners are
stored in a CSV (profiles/tunableop/), keyed and validated by the PyTorch,
HIP, hipBLASLt and rocBLAS versions and the GPU arch, and replayed with tuning
OFF -- no run-time search, no effect on shapes that are not in the file.

  mode "use"  : load the committed file (if its validators match) -- default
  mode "tune" : time every new GEMM shape and write the file at exit
  mode "off"  : library defaults
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Optional

import torch

ROOT = Path(__file__).resolve().parents[2]
TUNING_DIR = ROOT / "profiles" / "tunableop"


def default_file(model: str) -> Path:
    return TUNING_DIR / f"{model}_gfx950.csv"


def configure(mode: str, model: str, path: Optional[str] = None) -> Optional[str]:
    """Set up TunableOp for this process.  Returns the results file in use (or None)."""
    if mode == "off" or not torch.cuda.is_available():
        return None
    tun = torch.cuda.tunable
    f = Path(path) if path else default_file(model)
    if mode == "use":
        if not f.exists():
            return None
        tun.enable(True)
        tun.tuning_enable(False)
        tun.record_untuned_enable(False)
        # set_filename before enable() would make torch also WRITE to the file at
        # exit; read it explicitly instead and leave the committed file untouched
        tun.set_filename(str(Path(os.environ.get("TMPDIR", "/tmp")) / f"dmp_tunableop_{os.getpid()}.csv"))
        tun.read_file(str(f))
        return str(f)
    if mode == "tune":
        f.parent.mkdir(parents=True, exist_ok=True)
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(100)
        tun.set_max_tuning_iterations(30)
        tun.set_filename(str(f))  # TunableOp writes the results file at process exit
        return str(f)
    raise ValueError(f"unknown gemm tuning mode {mode!r}")
