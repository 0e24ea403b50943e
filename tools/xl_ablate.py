#!/usr/bin/env python3
"""gemm_xl ablation timings (interleaved rounds in one process): full ring
pipeline vs no in-loop copies / no fragment reads / MFMAs only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _C as C  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    dims = [int(x) for x in sys.argv[1:]] or [8192]
    m, n, k = (dims * 3)[:3] if len(dims) == 1 else dims
    a = torch.rand(m, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
    b = torch.rand(n, k, device="cuda", dtype=torch.bfloat16) * 2 - 1
    names = {(0, 4): "4-phase", (1, 4): "ring gm4", (1, 1): "ring gm1", (1, 2): "ring gm2",
             (1, 8): "ring gm8", (2, 4): "ring-nocopy", (3, 4): "ring-noread", (4, 4): "mfma-only", (5, 4): "no-epilogue", (6, 4): "persistent", (6, 8): "persist gm8",
             (6, 2): "persist gm2"}
    res = {p: [] for p in names}
    for _ in range(5):
        for p in names:
            C.set_gemm_xl_bn(int(os.environ.get('XL_BN', '256')), p[0], p[1])
            res[p].append(timeit(lambda: C.gemm_xl(a, b)))
    C.set_gemm_xl_bn(0, 1)
    fl = 2.0 * m * n * k
    for p, v in res.items():
        v.sort()
        print(f"{names[p]:12s} median {v[2]:.3f} ms  min {v[0]:.3f}  {fl / v[2] / 1e9:.0f} TF/s")


if __name__ == "__main__":
    main()
