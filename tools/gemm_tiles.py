#!/usr/bin/env python3
"""Sweep the NT GEMM tile variants (set_gemm_tile) over the ResNet-50 bs256
1x1-conv shapes: forward with BN moments, data gradient with the fused
shortcut add, plain store.  HIP-event timing; prints ms and achieved TB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from tools.microbench import timeit  # noqa: E402

C = _native.require("gemm tiles")
dev, dt = "cuda", torch.bfloat16
NAMES = {-1: "auto", 0: "256x64", 1: "128x64", 2: "128x128", 3: "128x64w", 4: "64x128", 5: "64x64",
         6: "256x128w8"}
shapes = [  # M, N(out), K(in), mode
    (802816, 256, 64, "moments"), (802816, 64, 256, "moments"), (802816, 256, 64, "add"),
    (200704, 512, 128, "moments"), (200704, 128, 512, "moments"), (200704, 512, 128, "add"),
    (50176, 1024, 256, "moments"), (50176, 256, 1024, "moments"), (50176, 1024, 256, "add"),
    (12544, 2048, 512, "moments"), (12544, 512, 2048, "moments"), (8192, 8192, 8192, "store"),
]
print(f"{'M':>7} {'N':>5} {'K':>5} {'mode':>8} | " + " ".join(f"{NAMES[t]:>9}" for t in NAMES) + "  (ms; best TB/s)")
for M, N, K, mode in shapes:
    a = torch.randn(M, K, device=dev, dtype=dt)
    w = torch.randn(N, K, device=dev, dtype=dt)
    r = torch.randn(M, N, device=dev, dtype=dt) if mode == "add" else None
    res = []
    for t in NAMES:
        C.set_gemm_tile(t)
        if mode == "add":
            ms = timeit(lambda: C.gemm_nt(a, w, mode="add", residual=r))
        else:
            ms = timeit(lambda: C.gemm_nt(a, w, mode=mode))
        res.append(ms)
    C.set_gemm_tile(-1)
    by = 2 * (M * K + M * N + (M * N if mode == "add" else 0))
    print(f"{M:7d} {N:5d} {K:5d} {mode:>8} | " + " ".join(f"{x:9.3f}" for x in res)
          + f"  {by / min(res) / 1e9:5.2f}")


# implicit-GEMM 3x3 conv forward per tile variant (ResNet-50 bs256 shapes)
from distributed_model_parallel_amd.ops.conv_igemm import _wmat  # noqa: E402
print(f"\n{'C':>4} {'H':>3} {'s':>2} | " + " ".join(f"{NAMES[t]:>9}" for t in NAMES) + "  (ms; best TF/s)")
for c, h, st in [(64, 56, 1), (128, 56, 2), (128, 28, 1), (256, 28, 2), (256, 14, 1), (512, 14, 2), (512, 7, 1)]:
    x = torch.randn(256, c, h, h, device=dev, dtype=dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device=dev, dtype=dt) * 0.05).contiguous(memory_format=torch.channels_last)
    ho = (h + 2 - 3) // st + 1
    res = []
    for t in NAMES:
        C.set_gemm_tile(t)
        res.append(timeit(lambda: C.conv_nt(x, _wmat(w), 3, 3, st, 1, ho, ho, mode="moments")))
    C.set_gemm_tile(-1)
    fl = 2 * 256 * ho * ho * c * c * 9
    print(f"{c:4d} {h:3d} {st:2d} | " + " ".join(f"{v:9.3f}" for v in res) + f"  {fl / min(res) / 1e9:7.1f}")
