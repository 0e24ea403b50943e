#!/usr/bin/env python3
"""Trimmed ping-pong tiles (gemm_xl.hip pick_bm) against 256-row tiles, on
the MFMA-bound shapes whose last round of 256-row tiles is partly empty:
ResNet-50's layer-3/4 3x3 convolutions (forward with BN moments, data
gradient with the BN backward) at batch 2048, and ViT-B/16's N = 768 GEMMs
at batch 256 (against hipBLASLt too).  Interleaved rounds, HIP events.

usage: python tools/xl_bm_bench.py [--reps 20] [--rounds 3]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_model_parallel_amd import _native  # noqa: E402

CL = torch.channels_last


def timeit(fn, reps):
    for _ in range(3):
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    C = _native.require("xl_bm_bench")
    dev = "cuda"
    cases = []
    for c, h in ((256, 14), (512, 7)):
        x = torch.randn(a.batch, c, h, h, device=dev).bfloat16().contiguous(memory_format=CL)
        w = (torch.randn(c, 9 * c, device=dev) * 0.03).bfloat16()
        y = torch.relu(torch.randn(a.batch * h * h, c, device=dev)).bfloat16()
        m = torch.zeros(c, device=dev)
        cases.append((f"conv_xl fwd moments {c}ch {h}x{h} b{a.batch}", (a.batch * h * h, c, 9 * c),
                      lambda x=x, w=w, h=h: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"), None))
        cases.append((f"conv_xl dgrad bnbwd_y {c}ch {h}x{h} b{a.batch}", (a.batch * h * h, c, 9 * c),
                      lambda x=x, w=w, h=h, y=y, m=m: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "bnbwd", bn_x=y, bn_y=y,
                                                                  mean=m), None))
    T = 256 * 197
    for name, n, k in (("qkv dgrad", 768, 2304), ("proj dgrad/fwd", 768, 768), ("fc1 dgrad / fc2 fwd", 768, 3072),
                       ("fc1 fwd", 3072, 768), ("qkv fwd", 2304, 768)):
        A = torch.randn(T, k, device=dev).bfloat16()
        B = (torch.randn(n, k, device=dev) * 0.03).bfloat16()
        cases.append((f"ViT {name} {T}x{n}x{k}", (T, n, k), lambda A=A, B=B: C.gemm_xl(A, B, "store"),
                      lambda A=A, B=B: torch.mm(A, B.t())))
    print("| shape | bm auto | 256-row ms | trimmed ms | gain | hipBLASLt ms | TF/s trimmed |")
    print("|---|---|---|---|---|---|---|")
    for name, (M, N, K), fn, lib in cases:
        C.set_gemm_xl_bm(0)
        bm = C.get_gemm_xl_bm(M, N, K)
        t256, tbm, tlib = [], [], []
        for _ in range(a.rounds):
            C.set_gemm_xl_bm(-1)
            t256.append(timeit(fn, a.reps))
            C.set_gemm_xl_bm(0)
            tbm.append(timeit(fn, a.reps))
            if lib is not None:
                tlib.append(timeit(lib, a.reps))
        x0, x1 = min(t256), min(tbm)
        tf = 2.0 * M * N * K / (x1 * 1e-3) / 1e12
        lb = f"{min(tlib):.4f}" if tlib else "-"
        print(f"| {name} | {bm} | {x0:.4f} | {x1:.4f} | {x0 / x1:.3f}x | {lb} | {tf:.0f} |", flush=True)
        torch.cuda.empty_cache()
    C.set_gemm_xl_bm(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
