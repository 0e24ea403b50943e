#!/usr/bin/env python3
"""Ping-pong TN weight gradient (gemm_tn_xl / conv_wgrad_xl) vs the split-M TN
kernel and MIOpen, sweeping the number of 256-block rounds the split count
targets.  ResNet-50 batch-1024 shapes.  HIP events, ms per call."""
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
    C = _native.require("tn xl bench")
    dt = torch.bfloat16
    print("| shape | tn (split-M) | MIOpen | xl r=0 | r=1 | r=2 | r=3 | r=4 | r=8 |")
    print("|---|---|---|---|---|---|---|---|---|")
    cases = [("l3 1x1 conv1 (1024->256)", 1024, 256, 14, 1), ("l4 1x1 conv1 (2048->512)", 2048, 512, 7, 1),
             ("l3 3x3 (256->256)", 256, 256, 14, 3), ("l4 3x3 (512->512)", 512, 512, 7, 3)]
    for name, cin, cout, h, k in cases:
        n = 1024
        x = torch.randn(n, cin, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(n, cout, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, cin, k, k, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        p = k // 2
        if k == 1:
            t_tn = timeit(lambda: C.gemm_tn(dy2, x2, dt))
            xl = lambda: C.gemm_tn_xl(dy2, x2, dt)  # noqa: E731
        else:
            t_tn = timeit(lambda: C.conv_wgrad(dy2, x, k, k, 1, p, h, h, dt))
            xl = lambda: C.conv_wgrad_xl(dy2, x, k, k, 1, p, h, h, dt)  # noqa: E731
        t_mi = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (p, p), (1, 1), False,
                                                                  (0, 0), 1, (False, True, False)))
        ts = []
        for r in (0, 1, 2, 3, 4, 8):
            C.set_tn_xl_rounds(r)
            ts.append(timeit(xl))
        C.set_tn_xl_rounds(0)
        print(f"| {name} | {t_tn:.3f} | {t_mi:.3f} | " + " | ".join(f"{t:.3f}" for t in ts) + " |", flush=True)


if __name__ == "__main__":
    torch.backends.cudnn.benchmark = True
    main()
