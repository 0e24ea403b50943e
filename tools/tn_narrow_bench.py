#!/usr/bin/env python3
"""A/B of the 4-wave weight-gradient kernel's narrow tiles (set_tn_narrow)
on the ResNet-50 batch-2048 1x1 weight-gradient shapes with a side of 64 or
128; interleaved rounds, median ms and effective TB/s (operands read once).

usage: python tools/tn_narrow_bench.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("tn narrow bench")
SHAPES = [  # name, M (rows), N (Cout), K (Cin)
    ("l1_c1", 6422528, 64, 256),
    ("l1_c1_b0", 6422528, 64, 64),
    ("l1_c3", 6422528, 256, 64),
    ("l2_c1_b0", 6422528, 128, 256),
    ("l2_c1", 1605632, 128, 512),
    ("l2_c3", 1605632, 512, 128),
    ("bs256_l1_c1", 802816, 64, 256),
    ("bs256_l1_c3", 802816, 256, 64),
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
    ops = []
    for name, M, N, K in SHAPES:
        a = torch.randn(M, N, device="cuda").bfloat16()
        b = torch.randn(M, K, device="cuda").bfloat16()
        ops.append((name, M * (N + K) * 2, lambda a=a, b=b: C.gemm_tn_xl(a, b, torch.float32)))
    res = {}
    for r in range(args.rounds):
        for name, by, fn in ops:
            for arm in ("narrow", "wide"):
                C.set_tn_narrow(arm == "narrow")
                res.setdefault((name, arm), []).append(timeit(fn, args.iters))
        print(f"round {r} done", flush=True)
    C.set_tn_narrow(True)
    print("| shape | arm | median ms | min ms | TB/s (operands once) |\n|---|---|---|---|---|")
    for name, by, _ in ops:
        for arm in ("narrow", "wide"):
            t = res[(name, arm)]
            med = statistics.median(t)
            print(f"| {name} | {arm} | {med:.4f} | {min(t):.4f} | {by / med / 1e9:.2f} |")


if __name__ == "__main__":
    main()
