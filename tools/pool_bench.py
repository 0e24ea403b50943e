"""Time the native NHWC max-pool forward/backward on the ResNet-50 stem shape.

    python tools/pool_bench.py [--batch 1024]

HIP-event timing over 20 launches after 3 warmups; prints ms and the
effective HBM rate of the bytes each kernel must move (fwd: x in, y + argmax
bytes out; bwd: dy + argmax in, dx out).
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_model_parallel_amd import _native  # noqa: E402


def _time(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    C = _native.require("pool_bench")
    x = torch.randn(args.batch, 64, 112, 112, device="cuda", dtype=torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    y, idx = C.maxpool2d_forward(x, 3, 2, 1)
    dy = torch.randn_like(y)
    tf = _time(lambda: C.maxpool2d_forward(x, 3, 2, 1))
    tb = _time(lambda: C.maxpool2d_backward(dy, idx, 112, 112, 3, 2, 1))
    fwd_bytes = x.numel() * 2 + y.numel() * 3
    bwd_bytes = dy.numel() * 3 + x.numel() * 2
    print(f"maxpool bs{args.batch}: fwd {tf:.3f} ms ({fwd_bytes / tf / 1e9:.2f} TB/s), "
          f"bwd {tb:.3f} ms ({bwd_bytes / tb / 1e9:.2f} TB/s)")


if __name__ == "__main__":
    main()
