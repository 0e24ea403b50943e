#!/usr/bin/env python3
"""Run one conv-epilogue GEMM configuration a few times for rocprofv3 --pmc
(one counter set per run).  SHAPE=name (from the table below), MODE=moments |
affine | affine_res | bnbwd | bnbwd_res, X2=0|2 (gemm_x2 kernel), ITERS=n.

usage: SHAPE=l2_conv3 MODE=affine_res rocprofv3 --pmc ... -- python3 tools/gemm_pmc_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

SHAPES = {  # (M, K, N) at ResNet-50 batch 256
    "l1_conv3": (802816, 64, 256), "l2_conv3": (200704, 128, 512), "l3_conv3": (50176, 256, 1024),
    "l4_conv3": (12544, 512, 2048), "l3_conv1": (50176, 1024, 256),
}


def main():
    C = _native.require("gemm pmc probe")
    M, K, N = SHAPES[os.environ.get("SHAPE", "l2_conv3")]
    mode = os.environ.get("MODE", "affine_res")
    C.set_gemm_xl_x2(int(os.environ.get("X2", "0")))
    torch.manual_seed(0)
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    sh = torch.randn(N, device="cuda")
    res = torch.randn(M, N, device="cuda").bfloat16()
    x = torch.randn(M, N, device="cuda").bfloat16()
    mean, inv, bb = x.float().mean(0), torch.rand(N, device="cuda") + 0.5, torch.randn(N, device="cuda")
    fns = {"moments": lambda: C.gemm_xl_conv(a, w, "moments"),
           "affine": lambda: C.gemm_xl_conv(a, w, "affine", shift=sh, relu=True),
           "affine_res": lambda: C.gemm_xl_conv(a, w, "affine", shift=sh, residual=res, relu=True),
           "bnbwd": lambda: C.gemm_xl_conv(a, w, "bnbwd", bn_x=x, mean=mean, invstd=inv, bias=bb),
           "bnbwd_res": lambda: C.gemm_xl_conv(a, w, "bnbwd", residual=res, bn_x=x, mean=mean, invstd=inv, bias=bb)}
    fn = fns[mode]
    for _ in range(int(os.environ.get("ITERS", 4))):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.environ.get('SHAPE', 'l2_conv3')} {mode} x2={os.environ.get('X2', '0')}: {e0.elapsed_time(e1):.4f} ms")


if __name__ == "__main__":
    main()
