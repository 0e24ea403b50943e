#!/usr/bin/env python3
"""3x3 weight gradients that are not on the halo kernel at 224 px (layer 4's
stride-2 first block, Cin = Cout = 512, 14 -> 7) and the halo-covered
neighbours, at batch 2048 and 256: MIOpen igemm_wrw vs the ping-pong TN
tap-gather kernel (conv_wgrad_xl) vs the halo kernel (wgrad3x3) where it
applies.  HIP events, ms per call."""
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
    C = _native.require("wgrad s2 bench")
    dt = torch.bfloat16
    print("| shape | batch | MIOpen | conv_wgrad_xl | halo wgrad3x3 |\n|---|---|---|---|---|")
    for n in (2048, 256):
        for name, c, hi, s in (("l4 s2 512 14->7", 512, 14, 2), ("l4 s1 512 7->7", 512, 7, 1),
                               ("l3 s2 256 28->14", 256, 28, 2), ("l3 s1 256 14->14", 256, 14, 1)):
            ho = (hi + 2 - 3) // s + 1
            x = torch.randn(n, c, hi, hi, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
            dy = torch.randn(n, c, ho, ho, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
            w = torch.randn(c, c, 3, 3, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, c)
            t_mi = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (s, s), (1, 1), (1, 1), False,
                                                                      (0, 0), 1, (False, True, False)))
            t_xl = timeit(lambda: C.conv_wgrad_xl(dy2, x, 3, 3, s, 1, ho, ho, dt))
            t_h = timeit(lambda: C.wgrad3x3(dy, x, s)) if C.wgrad3x3_supported(c, ho, ho, s) else float("nan")
            print(f"| {name} | {n} | {t_mi:.3f} | {t_xl:.3f} | {t_h:.3f} |", flush=True)
            del x, dy, w, dy2
            torch.cuda.empty_cache()


if __name__ == "__main__":
    torch.backends.cudnn.benchmark = True
    main()
