#!/usr/bin/env python3
"""A/B of the 4-wave GEMM's tile height (csrc/gemm/gemm_xl.hip
gemm_xl_w4_kernel MB = 8 / 7: 256- vs 224-row tiles) on the grids whose last
1-block/CU round is partial, plus hipBLASLt (torch.mm) on the plain ones.
Interleaved rounds in one process, random operands; median ms and TF/s.

usage: python tools/w4_trim_bench.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("w4 trim bench")
DEV = "cuda"

PLAIN = [  # name, M, N, K, mode
    ("vit_qkv_dgrad", 50432, 768, 2304, "store"),
    ("vit_proj_dgrad", 50432, 768, 768, "store"),
    ("vit_fc1_dgrad", 50432, 768, 3072, "store"),
    ("vit_fc2_fwd", 50432, 768, 3072, "bias_res"),
    ("vit_proj_fwd", 50432, 768, 768, "bias_res"),
    ("vit_fc1_fwd", 50432, 3072, 768, "bias_gelu"),
]
CONV = [  # name, N, C, H, Cout (3x3 / s1 / p1, moments)
    ("r50_l3_3x3", 2048, 256, 14, 256),
    ("r50_l4_3x3", 2048, 512, 7, 512),
]


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    C.set_gemm_xl_bn(256, 11)
    cases = []
    for name, M, N, K, mode in PLAIN:
        a = torch.randn(M, K, device=DEV).bfloat16()
        b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
        bt = b.t().contiguous().t()
        kw = {}
        if mode != "store":
            kw["bias"] = torch.randn(N, device=DEV).bfloat16()
        if mode == "bias_res":
            kw["residual"] = torch.randn(M, N, device=DEV).bfloat16()
        if mode == "bias_gelu":
            kw["aux"] = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        arms = {"w4_256": (256, lambda a=a, b=b, kw=kw, mode=mode: C.gemm_xl(a, b, mode, **kw)),
                "w4_224": (224, lambda a=a, b=b, kw=kw, mode=mode: C.gemm_xl(a, b, mode, **kw))}
        if mode == "store":
            arms["lib"] = (0, lambda a=a, bt=bt: a.mm(bt.t()))
        cases.append((name, 2.0 * M * N * K, arms))
    for name, n, c, h, co in CONV:
        x = torch.randn(n, c, h, h, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, 9 * c, device=DEV) * 0.03).bfloat16()
        f = lambda x=x, w=w, h=h: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments")
        cases.append((name, 2.0 * n * h * h * co * 9 * c, {"w4_256": (256, f), "w4_224": (224, f)}))
    res = {}
    for r in range(args.rounds):
        for name, fl, arms in cases:
            for arm, (bm, fn) in arms.items():
                C.set_gemm_xl_bm(bm if bm else 0)
                res.setdefault((name, arm), []).append(timeit(fn, args.iters))
        print(f"round {r} done", flush=True)
    C.set_gemm_xl_bm(0)
    C.set_gemm_xl_bn(0)
    print("| shape | arm | median ms | min ms | TF/s (median) |\n|---|---|---|---|---|")
    for name, fl, arms in cases:
        for arm in arms:
            t = res[(name, arm)]
            med = statistics.median(t)
            print(f"| {name} | {arm} | {med:.4f} | {min(t):.4f} | {fl / med / 1e9:.0f} |")


if __name__ == "__main__":
    main()
