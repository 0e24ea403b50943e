"""Helpers shared by every hipGraph capture site (DataParallel replicas,
pipeline stage slots, whole-step capture)."""
from __future__ import annotations

import contextlib
import gc

import torch


@contextlib.contextmanager
def no_gc_during_capture(device=None):
    """Collect garbage, synchronise, and keep Python's collector off for the
    duration: a collection inside a stream capture runs destructors of tensors
    / events left by earlier eager steps (side-stream frees, event destroys)
    while the stream is capturing -- it aborted the GPU suite once (round 5,
    DataParallel capture; ADVICE r5 for the pipeline's)."""
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize(device)
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()
