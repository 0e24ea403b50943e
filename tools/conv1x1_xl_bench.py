#!/usr/bin/env python3
"""1x1-conv GEMMs of ResNet-50 at batch 1024 with the conv epilogues: 4-wave NT
kernel vs the 8-wave glds-ring kernel (gemm_xl_conv).  Forward with BN
moments, data gradient with the BN-backward epilogue (mask from the BN
affine), plain "add" dgrad.  HIP events, ms per call."""
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
    C = _native.require("bench")
    B = 1024
    # (name, M, Cin, Cout) of the stride-1 1x1 convs
    convs = [("l1.conv1", B * 3136, 256, 64), ("l1.conv3", B * 3136, 64, 256),
             ("l2.conv1", B * 784, 512, 128), ("l2.conv3", B * 784, 128, 512),
             ("l3.conv1", B * 196, 1024, 256), ("l3.conv3", B * 196, 256, 1024),
             ("l4.conv1", B * 49, 2048, 512), ("l4.conv3", B * 49, 512, 2048),
             ("l2.b0.conv1", B * 3136, 256, 128), ("l3.b0.conv1", B * 784, 512, 256),
             ("l4.b0.conv1", B * 196, 1024, 512)]
    print("| conv | M | Cin | Cout | fwd+mom nt | fwd+mom xl ring | fwd+mom xl pp | dgrad bnbwd nt | "
          "dgrad bnbwd xl ring | dgrad bnbwd xl pp |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, M, cin, cout in convs:
        x = torch.randn(M, cin, device="cuda").bfloat16()
        w = (torch.randn(cout, cin, device="cuda") * 0.05).bfloat16()
        dy = torch.randn(M, cout, device="cuda").bfloat16()
        wt = w.t().contiguous()
        mean = torch.zeros(cin, device="cuda")
        inv = torch.ones(cin, device="cuda")
        f_nt = timeit(lambda: C.gemm_nt(x, w, mode="moments"))
        d_nt = timeit(lambda: C.gemm_nt_bnbwd(dy, wt, None, x, None, mean, inv, None, None))
        res = {}
        for pipe in (1, 10, 11):  # ring vs ping-pong vs 4-wave main loop (auto tile width)
            C.set_gemm_xl_bn(0, pipe)
            res[pipe] = (
                timeit(lambda: C.gemm_xl_conv(x, w, "moments")) if cout % 8 == 0 and cin % 64 == 0 else float("nan"),
                timeit(lambda: C.gemm_xl_conv(dy, wt, "bnbwd", bn_x=x, mean=mean, invstd=inv))
                if cout % 64 == 0 else float("nan"))
        C.set_gemm_xl_bn(0)
        print(f"| {name} | {M} | {cin} | {cout} | {f_nt:.3f} | {res[1][0]:.3f} | {res[7][0]:.3f} | {d_nt:.3f} | "
              f"{res[1][1]:.3f} | {res[7][1]:.3f} |", flush=True)
        del x, w, dy, wt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
