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


if __name__ == "__main__" and "--gemm" not in sys.argv:
    main()


def gemm_bench():
    """Our MFMA NT GEMM (1x1 conv) vs MIOpen conv vs hipBLASLt on ResNet-50 1x1 shapes."""
    from distributed_model_parallel_amd import _native
    C = _native.require("gemm bench")
    dev, dt = "cuda", torch.bfloat16
    shapes = [(802816, 256, 64), (802816, 64, 256), (200704, 512, 128), (200704, 128, 512),
              (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)]
    print(f"{'M':>7} {'N':>5} {'K':>5} | {'ours':>8} {'ours+mom':>8} {'miopen':>8} {'blaslt':>8}  ms | ours TB/s  TF/s")
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=dt)
        w = torch.randn(N, K, device=dev, dtype=dt)
        t_o = timeit(lambda: C.gemm_nt(a, w))
        t_m = timeit(lambda: C.gemm_nt(a, w, mode="moments"))
        x4 = a.view(M // 3136 if M % 3136 == 0 else 1, -1, 1, K) if False else None
        hw = {802816: 56, 200704: 28, 50176: 14, 12544: 7}[M]
        x = a.view(256, hw, hw, K).permute(0, 3, 1, 2)
        w4 = w.view(N, K, 1, 1).contiguous(memory_format=torch.channels_last)
        t_c = timeit(lambda: F.conv2d(x, w4))
        t_b = timeit(lambda: a @ w.t())
        by = 2 * (M * K + N * K + M * N)
        print(f"{M:7d} {N:5d} {K:5d} | {t_o:8.3f} {t_m:8.3f} {t_c:8.3f} {t_b:8.3f}     | {by / t_o / 1e9:6.2f} {2 * M * N * K / t_o / 1e9:7.1f}")


if __name__ == "__main__" and "--gemm" in sys.argv:
    gemm_bench()
