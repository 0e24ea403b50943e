#!/usr/bin/env python3
"""Per-op device timings with HIP events (no profiler attached), to compare
against rocprofv3 kernel traces of the same process.  Diagnostic only."""
from __future__ import annotations

import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.ops import batchnorm as bn  # noqa: E402


def timeit(fn, iters=30, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dev = "cuda"
    dt = torch.bfloat16
    cl = torch.channels_last
    res = {}
    x = torch.randn(256, 256, 56, 56, device=dev, dtype=dt).contiguous(memory_format=cl)
    w1 = torch.randn(64, 256, 1, 1, device=dev, dtype=dt).contiguous(memory_format=cl)
    res["conv1x1 256->64 @56 fwd"] = timeit(lambda: F.conv2d(x, w1))
    x3 = torch.randn(256, 64, 56, 56, device=dev, dtype=dt).contiguous(memory_format=cl)
    w3 = torch.randn(64, 64, 3, 3, device=dev, dtype=dt).contiguous(memory_format=cl)
    res["conv3x3 64->64 @56 fwd"] = timeit(lambda: F.conv2d(x3, w3, padding=1))
    a2 = x.permute(0, 2, 3, 1).reshape(-1, 256)
    wm = w1.view(64, 256)
    res["mm [802816x256]x[256x64] (same as 1x1)"] = timeit(lambda: a2 @ wm.t())
    m = torch.randn(8192, 8192, device=dev, dtype=dt)
    t = timeit(lambda: m @ m, iters=10)
    res["mm 8192^3"] = t
    res["mm 8192^3 TFLOPs"] = 2 * 8192 ** 3 / t / 1e9
    C = 64
    w = torch.ones(C, device=dev)
    b = torch.zeros(C, device=dev)
    rm = torch.zeros(C, device=dev)
    rv = torch.ones(C, device=dev)
    res["bn+relu fwd [256,64,56,56]"] = timeit(lambda: bn.batch_norm_act(x3, rm, rv, w, b, True, 0.1, 1e-5, relu=True))
    xr = x3.detach().requires_grad_()
    y = bn.batch_norm_act(xr, rm, rv, w, b, True, 0.1, 1e-5, relu=True)
    g = torch.randn_like(y)
    res["bn+relu bwd [256,64,56,56]"] = timeit(lambda: torch.autograd.grad(y, xr, g, retain_graph=True))
    copy_src = torch.empty(256 * 1024 * 1024, device=dev, dtype=torch.uint8)
    copy_dst = torch.empty_like(copy_src)
    t = timeit(lambda: copy_dst.copy_(copy_src))
    res["copy 256MiB GB/s"] = 2 * copy_src.numel() / t / 1e6
    for k, v in res.items():
        print(f"{k:45s} {v:10.3f}")


if __name__ == "__main__":
    main()
