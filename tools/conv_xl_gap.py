#!/usr/bin/env python3
"""Where the 3x3 implicit-GEMM convs (conv_xl) lose against the plain ping-pong
GEMM: the same M x N x K with A gathered per tap (conv_xl "store") vs A
materialised as a dense [M, K] matrix (gemm_xl "store", identical tile grid and
main loop), for the ResNet-50 layer-3/4 3x3 shapes at a given batch.  The gap
is what the gather costs; the plain GEMM's distance from 2.5 PF/s is what the
tile grid / main loop costs.  HIP events, ms per call.

usage: python tools/conv_xl_gap.py [--batch 2048]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    n = ap.parse_args().batch
    C = _native.require("conv_xl gap")
    dt = torch.bfloat16
    print(f"# conv_xl (gathered A) vs gemm_xl (dense A), ResNet-50 batch {n}, 1x MI355X\n")
    print("| shape | M | N | K | tiles | conv_xl ms | TF/s | gemm_xl ms | TF/s | conv/gemm |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, c, h in (("l3 3x3 256", 256, 14), ("l4 3x3 512", 512, 7), ("l2 3x3 128 (c128 halo in the step)", 128, 28)):
        x = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, 9 * c, device="cuda") * 0.02).to(dt)
        M, N, K = n * h * h, c, 9 * c
        t_c = timeit(lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "store"))
        a = torch.randn(M, K, device="cuda").to(dt)
        t_g = timeit(lambda: C.gemm_xl(a, w, "store"))
        fl = 2.0 * M * N * K
        tiles = ((M + 255) // 256) * ((N + 255) // 256)
        print(f"| {name} | {M} | {N} | {K} | {tiles} | {t_c:.4f} | {fl / t_c / 1e9:.0f} | {t_g:.4f} | "
              f"{fl / t_g / 1e9:.0f} | {t_c / t_g:.2f} |", flush=True)
        del x, w, a
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
