#!/usr/bin/env python3
"""The BN-folded bottleneck data gradient da = [dz | a] @ Bb^T + ebias with the
producer BN's backward in the epilogue (ops/bn_fold._FoldDgrad), on the NT
conv GEMM (gemm_nt_bnbwd) vs the ping-pong GEMM (gemm_xl_conv "bnbwd"), at
the ResNet-50 shapes of a given batch.  The routing rule (ops/conv1x1._xl)
predates the round-4 epilogue changes; this re-measures it.  HIP events, ms.

usage: python tools/fold_dgrad_ab.py [--batch 2048]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops import conv1x1  # noqa: E402


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
    C = _native.require("fold dgrad A/B")
    dt = torch.bfloat16
    print(f"# folded bottleneck dgrad + BN backward epilogue, ResNet-50 batch {n}, 1x MI355X\n")
    print("| stage | M | K (dz + a) | N | gemm_nt_bnbwd ms | gemm_xl_conv ms | nt/xl | rule picks |")
    print("|---|---|---|---|---|---|---|---|")
    for name, w, hw in (("l1", 64, 56), ("l2", 128, 28), ("l3", 256, 14), ("l4", 512, 7)):
        M = n * hw * hw
        dz = torch.randn(M, 4 * w, device="cuda").to(dt)
        a = torch.randn(M, w, device="cuda").to(dt)
        Bb = (torch.randn(w, 5 * w, device="cuda") * 0.02).to(dt)
        eb = torch.randn(w, device="cuda")
        x = torch.randn(M, w, device="cuda").to(dt)
        mean = torch.randn(w, device="cuda") * 0.1
        inv = torch.rand(w, device="cuda") + 0.5
        bw = torch.rand(w, device="cuda") + 0.5
        bb = torch.randn(w, device="cuda") * 0.1
        t_nt = timeit(lambda: C.gemm_nt_bnbwd(dz, Bb, None, x, None, mean, inv, bw, bb, a2=a, ebias=eb))
        t_xl = timeit(lambda: C.gemm_xl_conv(dz, Bb, "bnbwd", bn_x=x, mean=mean, invstd=inv, weight=bw, bias=bb,
                                             a2=a, ebias=eb))
        pick = "xl" if conv1x1._xl(w, 4 * w) else "nt"
        print(f"| {name} | {M} | {4 * w} + {w} | {w} | {t_nt:.4f} | {t_xl:.4f} | {t_nt / t_xl:.2f} | {pick} |",
              flush=True)
        del dz, a, Bb, x
        torch.cuda.empty_cache()
    print(f"\n# folded bottleneck forward (conv3 + bn3 affine + residual + ReLU), batch {n}\n")
    print("| stage | M | K | N | gemm_nt affine ms | gemm_xl_conv affine ms | nt/xl | rule picks |")
    print("|---|---|---|---|---|---|---|---|")
    for name, w, hw in (("l1", 64, 56), ("l2", 128, 28), ("l3", 256, 14), ("l4", 512, 7)):
        M = n * hw * hw
        a = torch.randn(M, w, device="cuda").to(dt)
        W = (torch.randn(4 * w, w, device="cuda") * 0.05).to(dt)
        sc = torch.rand(4 * w, device="cuda") + 0.5
        sh = torch.randn(4 * w, device="cuda") * 0.1
        res = torch.randn(M, 4 * w, device="cuda").to(dt)
        t_nt = timeit(lambda: C.gemm_nt(a, W, mode="affine", epi_scale=sc, epi_shift=sh, residual=res, relu=True))
        t_xl = timeit(lambda: C.gemm_xl_conv(a, W, "affine", residual=res, scale=sc, shift=sh, relu=True))
        pick = "xl" if conv1x1._xl(4 * w, w) else "nt"
        print(f"| {name} | {M} | {w} | {4 * w} | {t_nt:.4f} | {t_xl:.4f} | {t_nt / t_xl:.2f} | {pick} |", flush=True)
        del a, W, res
        torch.cuda.empty_cache()
    print(f"\n# bottleneck conv1 forward with BN moments (K = block input, N = width), batch {n}\n")
    print("| stage | M | K | N | gemm_nt moments ms | gemm_xl_conv moments ms | nt/xl | rule picks |")
    print("|---|---|---|---|---|---|---|---|")
    for name, w, hw in (("l1", 64, 56), ("l2", 128, 28), ("l3", 256, 14), ("l4", 512, 7)):
        M = n * hw * hw
        a = torch.randn(M, 4 * w, device="cuda").to(dt)
        W = (torch.randn(w, 4 * w, device="cuda") * 0.05).to(dt)
        t_nt = timeit(lambda: C.gemm_nt(a, W, mode="moments"))
        t_xl = timeit(lambda: C.gemm_xl_conv(a, W, "moments"))
        pick = "xl" if conv1x1._xl(w, 4 * w) else "nt"
        print(f"| {name} | {M} | {4 * w} | {w} | {t_nt:.4f} | {t_xl:.4f} | {t_nt / t_xl:.2f} | {pick} |", flush=True)
        del a, W
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
