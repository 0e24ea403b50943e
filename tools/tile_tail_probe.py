#!/usr/bin/env python3
"""What the partial last round of 256 x 256 tiles costs the layer-3/4 3x3
convs (conv_xl, one block per CU): time per image at batch 2048 (l3: 1568
tiles = 6.1 rounds of 256 CUs, l4: 784 = 3.06) against batches whose tile
count just fills whole rounds.  If the per-image time at 2048 is clearly
higher, splitting the last round's tiles over K (stream-K) would pay.
HIP events, ms per call.

usage: python tools/tile_tail_probe.py
"""
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
    C = _native.require("tile tail probe")
    dt = torch.bfloat16
    print("| conv | batch | tiles | rounds (256 CUs) | ms | us per image |")
    print("|---|---|---|---|---|---|")
    for name, c, h, batches in (("l3 3x3 256 @14", 256, 14, (2048, 2006, 1671, 1337)),
                                ("l4 3x3 512 @7", 512, 7, (2048, 2006, 1337))):
        w = (torch.randn(c, 9 * c, device="cuda") * 0.02).to(dt)
        for n in batches:
            x = torch.randn(n, c, h, h, device="cuda").to(dt).contiguous(memory_format=torch.channels_last)
            M = n * h * h
            tiles = ((M + 255) // 256) * ((c + 255) // 256)
            t = timeit(lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"))
            print(f"| {name} | {n} | {tiles} | {tiles / 256:.2f} | {t:.4f} | {1000 * t / n:.3f} |", flush=True)
            del x
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
