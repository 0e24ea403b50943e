#!/usr/bin/env python3
"""The fused stem BN + ReLU + max-pool kernels (csrc/pool/maxpool.hip
bnpool_fwd / bnpool_bwd) at the ResNet-50 stem shape, HIP events.

usage: python tools/pool_bn_bench.py [--batch 2048] [--reps 10]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, reps):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    C = _native.require("pool_bn_bench")
    n, c, h = a.batch, 64, 112
    x = torch.randn(n, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    sc = torch.rand(c, device="cuda") + 0.5
    sh = torch.randn(c, device="cuda") * 0.1
    mean = torch.randn(c, device="cuda") * 0.1
    y, idx = C.maxpool2d_bn_forward(x, sc, sh, 3, 2, 1)
    dy = torch.randn_like(y)
    tf = timeit(lambda: C.maxpool2d_bn_forward(x, sc, sh, 3, 2, 1), a.reps)
    tb = timeit(lambda: C.maxpool2d_bn_backward(dy, idx, x, sc, sh, mean, 3, 2, 1), a.reps)
    xb = x.numel() * 2
    fwd_bytes = xb + y.numel() * 2 + idx.numel()
    bwd_bytes = dy.numel() * 2 + idx.numel() + 2 * xb
    print(f"| kernel | ms | unique GB | TB/s |\n|---|---|---|---|")
    print(f"| bnpool forward | {tf:.3f} | {fwd_bytes / 1e9:.2f} | {fwd_bytes / tf / 1e9:.2f} |")
    print(f"| bnpool backward | {tb:.3f} | {bwd_bytes / 1e9:.2f} | {bwd_bytes / tb / 1e9:.2f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
