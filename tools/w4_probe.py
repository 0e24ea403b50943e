#!/usr/bin/env python3
"""Run one 8192^3-class NT GEMM arm a few times for rocprofv3 --pmc (one
counter set per run): ARM = w4 | lib | xl, VAR = gemm_w4 variant, SIZE = n.

usage: ARM=w4 VAR=4 rocprofv3 --pmc ... -- python3 tools/w4_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def main():
    C = _native.require("w4 probe")
    n = int(os.environ.get("SIZE", "8192"))
    arm = os.environ.get("ARM", "w4")
    var = int(os.environ.get("VAR", "4"))
    torch.manual_seed(0)
    a = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    b = torch.rand(n, n, device="cuda", dtype=torch.bfloat16) * 2 - 1
    if arm == "w4":
        fn = lambda: C.gemm_w4(a, b, 0, var)  # noqa: E731
    elif arm == "lib":
        fn = lambda: a @ b.t()  # noqa: E731
    else:
        C.set_gemm_xl_bn(256, 10, 0)
        fn = lambda: C.gemm_xl(a, b)  # noqa: E731
    for _ in range(int(os.environ.get("ITERS", "6"))):
        fn()
    torch.cuda.synchronize()
    print(f"{arm} var={var} n={n} done", flush=True)


if __name__ == "__main__":
    main()
