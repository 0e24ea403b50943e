#!/usr/bin/env python3
"""A/B of the short-K conv-epilogue GEMMs: gemm_xl ring kernel (one 256x256
block per CU) vs gemm_x2_kernel (two 256x128 blocks per CU, register
epilogue) on the ResNet-50 1x1-conv shapes at batch 256 per GPU.  HIP events,
ms per call, next to the HBM roofline bound (operands and results moved
once at 8 TB/s; MFMA at 2.5 PF/s when larger).

usage: python tools/x2_bench.py [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, iters=20):
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
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    C = _native.require("x2 bench")
    n = args.batch
    # (name, pixels, K, N): forward conv3 (moments / affine), forward conv1
    # of the next block, and the conv3 data gradient (bnbwd, K = Cout)
    shapes = [("l1 conv3", n * 56 * 56, 64, 256), ("l2 conv3", n * 28 * 28, 128, 512),
              ("l2 conv1", n * 28 * 28, 512, 128), ("l3 conv3", n * 14 * 14, 256, 1024),
              ("l3 conv1", n * 14 * 14, 1024, 256), ("l4 conv3", n * 7 * 7, 512, 2048),
              ("l4 conv1", n * 7 * 7, 2048, 512), ("l1 dgrad1", n * 56 * 56, 64, 256),
              ("l2 dgrad1", n * 28 * 28, 128, 512), ("l3 dgrad1", n * 14 * 14, 256, 1024),
              ("l4 dgrad1", n * 7 * 7, 512, 2048)]
    old = C.get_gemm_xl_x2()
    print(f"# gemm_xl vs gemm_x2 conv epilogues, ResNet-50 batch {n}, 1x MI355X\n")
    print("| shape | M | K | N | mode | xl ms | x2 ms | xl/x2 | bound ms | x2 frac |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, M, K, N in shapes:
        torch.manual_seed(0)
        a = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        sh = torch.randn(N, device="cuda")
        res = torch.randn(M, N, device="cuda").bfloat16()
        io = 2 * (M * K + N * K + M * N)
        if "dgrad" in name:
            x = torch.randn(M, N, device="cuda").bfloat16()
            mean, inv, bb = x.float().mean(0), torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda")
            modes = {"bnbwd": (lambda: C.gemm_xl_conv(a, w, "bnbwd", bn_x=x, mean=mean, invstd=inv, bias=bb),
                               io + 2 * M * N),
                     "bnbwd+res": (lambda: C.gemm_xl_conv(a, w, "bnbwd", residual=res, bn_x=x, mean=mean,
                                                          invstd=inv, bias=bb), io + 4 * M * N)}
        else:
            modes = {"moments": (lambda: C.gemm_xl_conv(a, w, "moments"), io),
                     "affine": (lambda: C.gemm_xl_conv(a, w, "affine", shift=sh, relu=True), io),
                     "affine+res": (lambda: C.gemm_xl_conv(a, w, "affine", shift=sh, residual=res, relu=True),
                                    io + 2 * M * N),
                     "add": (lambda: C.gemm_xl_conv(a, w, "add", residual=res), io + 2 * M * N)}
        for mode, (fn, nbytes) in modes.items():
            C.set_gemm_xl_x2(0)
            t0 = timeit(fn)
            C.set_gemm_xl_x2(2)
            t1 = timeit(fn)
            bound = 1e3 * max(2.0 * M * N * K / 2.5e15, nbytes / 8e12)
            print(f"| {name} | {M} | {K} | {N} | {mode} | {t0:.4f} | {t1:.4f} | {t0 / t1:.2f} | {bound:.4f} | "
                  f"{bound / t1:.0%} |", flush=True)
        del a, w, res
        torch.cuda.empty_cache()
    C.set_gemm_xl_x2(old)


if __name__ == "__main__":
    main()
