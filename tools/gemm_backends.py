#!/usr/bin/env python3
"""bf16 GEMM backends side by side on one process (HIP events, random operands):
our 4-wave NT kernel (csrc/conv/gemm_bf16.hip ``gemm_nt``), the 8-wave
256-row glds-ring kernel (csrc/gemm/gemm_xl.hip ``gemm_xl``) and hipBLASLt
(``torch.mm`` with the tuned solutions in effect).  Shapes: square sizes, the
ViT-B/16 linears at batch 256 (197 tokens) and the ResNet-50 implicit-GEMM
shapes at batch 1024 taken as plain GEMMs.  Markdown table on stdout.

usage: python tools/gemm_backends.py [comma-separated shape-name prefixes]
"""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


SHAPES = [
    ("square", 8192, 8192, 8192), ("square", 4096, 4096, 4096),
    ("vit qkv fwd", 50432, 2304, 768), ("vit proj fwd", 50432, 768, 768),
    ("vit fc1 fwd", 50432, 3072, 768), ("vit fc2 fwd", 50432, 768, 3072),
    ("vit fc1 dgrad", 50432, 768, 3072), ("vit qkv dgrad", 50432, 768, 2304),
    ("r50 l1 3x3 (as GEMM)", 3211264, 64, 576), ("r50 l2 3x3", 802816, 128, 1152),
    ("r50 l3 3x3", 200704, 256, 2304), ("r50 l4 3x3", 50176, 512, 4608),
    ("r50 l3 conv3 1x1", 200704, 1024, 256), ("r50 l4 conv1 1x1", 50176, 512, 2048),
]


def main():
    C = _native.require("gemm backends")
    dev, dt = "cuda", torch.bfloat16
    only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
    print("| shape | M | N | K | gemm_nt ms | gemm_xl ms | xl ping-pong ms | hipBLASLt ms | best TF/s | pp / blaslt |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, M, N, K in SHAPES:
        if only and not any(name.startswith(o) for o in only):
            continue
        a = torch.rand(M, K, device=dev, dtype=dt) * 2 - 1
        b = torch.rand(N, K, device=dev, dtype=dt) * 2 - 1
        t_nt = timeit(lambda: C.gemm_nt(a, b))
        t_xl = timeit(lambda: C.gemm_xl(a, b)) if (K % 64 == 0 and N % 8 == 0) else float("nan")
        t_pp = float("nan")
        if K % 64 == 0 and N % 8 == 0:
            C.set_gemm_xl_bn(256, 10)  # 256 x 256 8-wave ping-pong schedule (PIPE 10)
            try:
                t_pp = timeit(lambda: C.gemm_xl(a, b))
                err = (C.gemm_xl(a, b).float() - (a.float() @ b.float().t())).abs().max().item() if M * N <= 1 << 26 else 0.0
            finally:
                C.set_gemm_xl_bn(0)
            if err > 0.05 * K ** 0.5:
                print(f"  !! ping-pong max error {err:.3f}", flush=True)
        t_bl = timeit(lambda: a @ b.t())
        fl = 2.0 * M * N * K
        best = min(t for t in (t_nt, t_xl, t_pp, t_bl) if t == t)
        print(f"| {name} | {M} | {N} | {K} | {t_nt:.3f} | {t_xl:.3f} | {t_pp:.3f} | {t_bl:.3f} | {fl / best / 1e9:.0f} | "
              f"{t_pp / t_bl:.2f} |", flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
