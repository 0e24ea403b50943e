#!/usr/bin/env python3
"""Does a data gradient (epilogue-heavy, HBM-latency bound) overlap with the
weight gradient of the same layer (MFMA / L2 bound) when the two run on two
HIP streams?  ResNet-50 conv1 of layers 1-4 at batch 2048: sequential vs
concurrent, ms per pair."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from tools.fold_bench import timeit  # noqa: E402


def main():
    C = _native.require("bench")
    B = 2048
    side = torch.cuda.Stream()
    print("| conv1 | dgrad | wgrad | sequential | two streams | saved |")
    print("|---|---|---|---|---|---|")
    for name, M, cin, planes in [("l1", B * 3136, 256, 64), ("l2", B * 784, 512, 128), ("l3", B * 196, 1024, 256),
                                 ("l4", B * 49, 2048, 512)]:
        x = torch.relu(torch.randn(M, cin, device="cuda")).bfloat16()      # block input (conv1 input)
        dy = torch.randn(M, planes, device="cuda").bfloat16()              # grad at conv1 output
        wt = (torch.randn(cin, planes, device="cuda") * 0.05).bfloat16()  # W^T
        R = torch.randn(M, cin, device="cuda").bfloat16()
        xl = cin >= 512 or (cin >= 256 and planes <= 512)

        def dgrad():
            if xl:
                return C.gemm_xl_conv(dy, wt, "bnbwd", residual=R, bn_y=x)
            return C.gemm_nt_bnbwd(dy, wt, R, None, x, None, None, None, None)

        def wgrad():
            return C.gemm_tn_xl(dy, x, torch.bfloat16) if (planes >= 256 and cin >= 256 and M >= 150_000) \
                else C.gemm_tn(dy, x, torch.bfloat16)

        def both():
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(side):
                side.wait_event(ev)
                wgrad()
            dgrad()
            torch.cuda.current_stream().wait_stream(side)

        td, tw = timeit(dgrad), timeit(wgrad)
        ts = timeit(lambda: (dgrad(), wgrad()))
        tc = timeit(both)
        print(f"| {name} | {td:.3f} | {tw:.3f} | {ts:.3f} | {tc:.3f} | {100 * (ts - tc) / ts:.0f} % |", flush=True)
        del x, dy, wt, R


if __name__ == "__main__":
    main()
