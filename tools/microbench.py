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


if __name__ == "__main__" and not {"--gemm", "--conv", "--wgrad"} & set(sys.argv):
    main()


def gemm_bench():
    """Our MFMA NT GEMM (1x1 conv) vs MIOpen conv vs hipBLASLt on ResNet-50 1x1 shapes."""
    from distributed_model_parallel_amd import _native
    C = _native.require("gemm bench")
    dev, dt = "cuda", torch.bfloat16
    shapes = [(8192, 8192, 8192), (802816, 64, 576), (200704, 128, 1152), (50176, 256, 2304),
              (802816, 256, 64), (802816, 64, 256), (200704, 512, 128), (200704, 128, 512),
              (50176, 1024, 256), (50176, 256, 1024), (12544, 2048, 512), (12544, 512, 2048)]
    print(f"{'M':>7} {'N':>5} {'K':>5} | {'ours':>8} {'ours+mom':>8} {'miopen':>8} {'blaslt':>8}  ms | ours TB/s  TF/s")
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=dt)
        w = torch.randn(N, K, device=dev, dtype=dt)
        t_o = timeit(lambda: C.gemm_nt(a, w))
        t_m = timeit(lambda: C.gemm_nt(a, w, mode="moments"))
        hw = {802816: 56, 200704: 28, 50176: 14, 12544: 7}.get(M)
        t_c = float("nan")
        if hw:
            x = a.view(256, hw, hw, K).permute(0, 3, 1, 2)
            w4 = w.view(N, K, 1, 1).contiguous(memory_format=torch.channels_last)
            t_c = timeit(lambda: F.conv2d(x, w4))
        t_b = timeit(lambda: a @ w.t())
        by = 2 * (M * K + N * K + M * N)
        print(f"{M:7d} {N:5d} {K:5d} | {t_o:8.3f} {t_m:8.3f} {t_c:8.3f} {t_b:8.3f}     | {by / t_o / 1e9:6.2f} {2 * M * N * K / t_o / 1e9:7.1f}")


def conv_bench():
    """Implicit-GEMM 3x3 conv (ours) vs MIOpen on the ResNet-50 bs256 3x3 shapes:
    forward, data gradient, weight gradient."""
    from distributed_model_parallel_amd import _native
    from distributed_model_parallel_amd.ops.conv_igemm import _wmat
    C = _native.require("conv bench")
    dev, dt, cl = "cuda", torch.bfloat16, torch.channels_last
    shapes = [(64, 56, 1), (128, 56, 2), (128, 28, 1), (256, 28, 2), (256, 14, 1), (512, 14, 2), (512, 7, 1)]
    print(f"{'C':>4} {'H':>3} {'s':>2} | {'fwd':>7} {'miopen':>7} | {'dgrad':>7} {'miopen':>7} | {'wgrad':>7} {'miopen':>7} ms | fwd TF/s")
    for c, h, s in shapes:
        x = torch.randn(256, c, h, h, device=dev, dtype=dt).contiguous(memory_format=cl)
        w = (torch.randn(c, c, 3, 3, device=dev, dtype=dt) * 0.05).contiguous(memory_format=cl)
        ho = (h + 2 - 3) // s + 1
        dy = torch.randn(256, c, ho, ho, device=dev, dtype=dt).contiguous(memory_format=cl)
        t_f = timeit(lambda: C.conv_nt(x, _wmat(w), 3, 3, s, 1, ho, ho))
        t_fm = timeit(lambda: F.conv2d(x, w, None, s, 1))
        wt = w.permute(1, 2, 3, 0).reshape(c, -1).contiguous()
        t_d = timeit(lambda: C.conv_nt(dy, wt, 3, 3, s, 1, h, h, transposed=True))
        t_dm = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (1, 1), (1, 1), False, (0, 0), 1, (True, False, False)))
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, c)
        t_w = timeit(lambda: C.conv_wgrad(dy2, x, 3, 3, s, 1, ho, ho, dt))
        t_wm = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (1, 1), (1, 1), False, (0, 0), 1, (False, True, False)))
        fl = 2 * 256 * ho * ho * c * c * 9
        print(f"{c:4d} {h:3d} {s:2d} | {t_f:7.3f} {t_fm:7.3f} | {t_d:7.3f} {t_dm:7.3f} | {t_w:7.3f} {t_wm:7.3f}    | {fl / t_f / 1e9:7.1f}")


if __name__ == "__main__" and "--gemm" in sys.argv:
    gemm_bench()
if __name__ == "__main__" and "--conv" in sys.argv:
    conv_bench()


def wgrad_bench():
    """1x1-conv weight / data gradients: our TN / NT kernels vs hipBLASLt (torch.mm)
    at every ResNet-50 bs256 1x1 shape -- the data behind ops/conv1x1.py's
    per-shape backend choice."""
    from distributed_model_parallel_amd import _native
    C = _native.require("wgrad bench")
    dev, dt = "cuda", torch.bfloat16
    # (M, Cin, Cout) of every distinct 1x1 conv in ResNet-50 at batch 256
    convs = [(802816, 64, 64), (802816, 64, 256), (802816, 256, 64), (200704, 256, 128),
             (200704, 128, 512), (200704, 512, 128), (50176, 512, 256), (50176, 256, 1024),
             (50176, 1024, 256), (12544, 1024, 512), (12544, 512, 2048), (12544, 2048, 512),
             (200704, 256, 512), (50176, 512, 1024), (12544, 1024, 2048)]
    print(f"{'M':>7} {'Cin':>5} {'Cout':>5} | {'wgrad ours':>10} {'blaslt':>8} | {'dgrad ours':>10} {'blaslt':>8} ms")
    for M, cin, cout in convs:
        x = torch.randn(M, cin, device=dev, dtype=dt)
        dy = torch.randn(M, cout, device=dev, dtype=dt)
        w = torch.randn(cout, cin, device=dev, dtype=dt)
        wt = w.t().contiguous()
        t_w = timeit(lambda: C.gemm_tn(dy, x, dt))
        t_wb = timeit(lambda: dy.t() @ x)
        t_d = timeit(lambda: C.gemm_nt(dy, wt))
        t_db = timeit(lambda: dy @ w)
        print(f"{M:7d} {cin:5d} {cout:5d} | {t_w:10.3f} {t_wb:8.3f} | {t_d:10.3f} {t_db:8.3f}")


if __name__ == "__main__" and "--wgrad" in sys.argv:
    wgrad_bench()
