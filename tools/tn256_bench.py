#!/usr/bin/env python3
"""1x1-conv weight gradients of ResNet-50 at a given batch (default 256 per
GPU): the split-M 4-wave TN kernel (gemm_tn) vs the ping-pong TN kernel
(gemm_tn_xl) at its automatic split and at fixed split-round targets.
HIP events, ms per call; prints the conv1x1 routing rule's pick.

usage: python tools/tn256_bench.py [--batch 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops import conv1x1  # noqa: E402


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
    n = ap.parse_args().batch
    C = _native.require("tn256 bench")
    dt = torch.bfloat16
    # (name, pixels, Cout (dy columns), Cin (x columns)), dW = dy^T x
    cases = [("l1 conv1 64<-256", 56 * 56, 64, 256), ("l1 conv3 256<-64", 56 * 56, 256, 64),
             ("l1 ds 256<-64", 56 * 56, 256, 64), ("l2 conv1 128<-512", 28 * 28, 128, 512),
             ("l2 conv3 512<-128", 28 * 28, 512, 128), ("l2 ds 512<-256", 28 * 28, 512, 256),
             ("l3 conv1 256<-1024", 14 * 14, 256, 1024), ("l3 conv3 1024<-256", 14 * 14, 1024, 256),
             ("l3 ds 1024<-512", 14 * 14, 1024, 512), ("l4 conv1 512<-2048", 7 * 7, 512, 2048),
             ("l4 conv3 2048<-512", 7 * 7, 2048, 512), ("l4 ds 2048<-1024", 7 * 7, 2048, 1024)]
    print(f"# 1x1 weight gradients, ResNet-50 batch {n}, 1x MI355X\n")
    print("| shape | M | tn | tn_xl auto | r=1 | r=2 | r=4 | hipBLASLt | best/tn | rule picks |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, px, cout, cin in cases:
        m = n * px
        dy = torch.randn(m, cout, device="cuda").to(dt)
        x = torch.randn(m, cin, device="cuda").to(dt)
        t_tn = timeit(lambda: C.gemm_tn(dy, x, dt))
        ts = []
        for r in (0, 1, 2, 4):
            C.set_tn_xl_rounds(r)
            ts.append(timeit(lambda: C.gemm_tn_xl(dy, x, dt)))
        C.set_tn_xl_rounds(0)
        t_lib = timeit(lambda: dy.t().mm(x))
        pick = "tn_xl" if conv1x1._tn_xl(m, cout, cin) else "tn"
        print(f"| {name} | {m} | {t_tn:.4f} | " + " | ".join(f"{t:.4f}" for t in ts) +
              f" | {t_lib:.4f} | {min(ts) / t_tn:.2f} | {pick} |", flush=True)
        del dy, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
