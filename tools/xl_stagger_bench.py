#!/usr/bin/env python3
"""First-round phase stagger of the ping-pong GEMM (gemm_xl.hip, PIPE 7,
set_gemm_xl_stagger / DMP_XL_STAGGER): the ResNet-50 batch-2048 1x1 GEMMs
(short K: staging and an HBM-bound epilogue per tile) and a 3x3 implicit
GEMM, for several stagger delays, interleaved rounds in one process.

usage: python tools/xl_stagger_bench.py [--ticks 0 300 600 900] [--reps 10] [--rounds 3]
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
    ap.add_argument("--ticks", type=int, nargs="+", default=[0, 300, 600, 900])
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    C = _native.require("xl_stagger_bench")
    dev, bf = "cuda", torch.bfloat16
    cases = []
    for name, hw, w in (("l2", 28 * 28, 128), ("l3", 14 * 14, 256), ("l4", 7 * 7, 512)):
        M = a.batch * hw
        x = torch.randn(M, w, device=dev, dtype=bf)
        B = (torch.randn(4 * w, w, device=dev) * 0.05).to(bf)
        R = torch.randn(M, 4 * w, device=dev, dtype=bf)
        sc = torch.rand(4 * w, device=dev) + 0.5
        sh = torch.randn(4 * w, device=dev) * 0.1
        cases.append((f"{name} fwd affine+res+relu {M}x{4 * w}x{w}",
                      lambda x=x, B=B, R=R, sc=sc, sh=sh: C.gemm_xl_conv(x, B, "affine", residual=R, scale=sc,
                                                                        shift=sh, relu=True)))
        cases.append((f"{name} fwd moments {M}x{4 * w}x{w}", lambda x=x, B=B: C.gemm_xl_conv(x, B, "moments")))
        if w >= 256:
            dz = torch.randn(M, 4 * w, device=dev, dtype=bf)
            a2 = torch.randn(M, w, device=dev, dtype=bf)
            Bb = (torch.randn(w, 5 * w, device=dev) * 0.03).to(bf)
            eb = torch.randn(w, device=dev) * 0.1
            y = torch.relu(torch.randn(M, w, device=dev)).to(bf)
            cases.append((f"{name} fold dgrad bnbwd(y) {M}x{w}x{5 * w}",
                          lambda dz=dz, Bb=Bb, a2=a2, eb=eb, y=y: C.gemm_xl_conv(dz, Bb, "bnbwd", bn_y=y, a2=a2,
                                                                                ebias=eb)))
    xs = torch.randn(a.batch, 256, 14, 14, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
    ws = (torch.randn(256, 9 * 256, device=dev) * 0.03).to(bf)
    cases.append(("l3 3x3 conv_xl moments", lambda: C.conv_xl(xs, ws, 3, 3, 1, 1, 14, 14, "moments")))
    print("| GEMM | " + " | ".join(f"{t} ticks ms" for t in a.ticks) + " | best gain |")
    print("|---|" + "---|" * len(a.ticks) + "---|")
    for name, fn in cases:
        res = {t: [] for t in a.ticks}
        for _ in range(a.rounds):
            for t in a.ticks:
                C.set_gemm_xl_stagger(t)
                res[t].append(timeit(fn, a.reps))
        best = {t: min(v) for t, v in res.items()}
        gain = best[a.ticks[0]] / min(best.values())
        print(f"| {name} | " + " | ".join(f"{best[t]:.4f}" for t in a.ticks) + f" | {gain:.3f}x |", flush=True)
    C.set_gemm_xl_stagger(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
