#!/usr/bin/env python3
"""Epilogue-heavy 1x1-conv GEMMs of ResNet-50 at batch 2048 (short K, wide N):
the next block's conv1 data gradient with the previous BN's fused backward
(mask from the block output y, shortcut gradient R added) and the folded
conv3 forward (affine + residual + ReLU).  4-wave NT kernel (2 blocks/CU)
vs the 8-wave ping-pong kernel (1 block/CU), ms per call and achieved TB/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from tools.fold_bench import timeit  # noqa: E402


def main():
    C = _native.require("bench")
    B = 2048
    print("| shape | M | K | N | bnbwd nt | bnbwd xl | TB/s best | affine nt | affine xl | TB/s best |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, M, K, N in [("l1", B * 3136, 64, 256), ("l2", B * 784, 128, 512), ("l3", B * 196, 256, 1024),
                          ("l4", B * 49, 512, 2048)]:
        dy = torch.randn(M, K, device="cuda").bfloat16()
        wt = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
        R = torch.randn(M, N, device="cuda").bfloat16()
        y = torch.relu(torch.randn(M, N, device="cuda")).bfloat16()
        b_nt = timeit(lambda: C.gemm_nt_bnbwd(dy, wt, R, None, y, None, None, None, None))
        b_xl = timeit(lambda: C.gemm_xl_conv(dy, wt, "bnbwd", residual=R, bn_y=y))
        gb = (M * K + 3 * M * N) * 2 / 1e9
        sc = torch.rand(N, device="cuda") + 0.5
        sh = torch.randn(N, device="cuda")
        a_nt = timeit(lambda: C.gemm_nt(dy, wt, mode="affine", epi_scale=sc, epi_shift=sh, residual=R, relu=True))
        a_xl = timeit(lambda: C.gemm_xl_conv(dy, wt, "affine", residual=R, scale=sc, shift=sh, relu=True))
        ga = (M * K + 2 * M * N) * 2 / 1e9
        print(f"| {name} | {M} | {K} | {N} | {b_nt:.3f} | {b_xl:.3f} | {gb / min(b_nt, b_xl):.2f} | {a_nt:.3f} | "
              f"{a_xl:.3f} | {ga / min(a_nt, a_xl):.2f} |", flush=True)
        del dy, wt, R, y


if __name__ == "__main__":
    main()
