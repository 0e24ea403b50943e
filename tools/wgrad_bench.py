#!/usr/bin/env python3
"""Time the halo-tiled 3x3 weight gradient (csrc/conv/wgrad3x3.hip) against
MIOpen (find mode, seeded db) on ResNet-50's stride-1 3x3 shapes at batch N.
HIP events, median of 20 after 5 warm-up calls.  --loop K: only run the halo
kernel K times per shape (for rocprofv3 --pmc passes).

  python tools/wgrad_bench.py [--batch 2048] [--only 64,128] [--loop 0]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.utils import miopen_db  # noqa: E402

SHAPES = [(64, 56, 1), (128, 28, 1), (256, 14, 1), (512, 7, 1), (128, 28, 2), (256, 14, 2)]


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--only", default="")
    ap.add_argument("--loop", type=int, default=0)
    args = ap.parse_args()
    only = [int(c) for c in args.only.split(",") if c]
    torch.backends.cudnn.benchmark = True
    miopen_db.seed("use")
    C = _native.require("wgrad_bench")
    print(f"3x3/s1 weight gradient, batch {args.batch}, ms per call (median of 20)")
    print("| C | out HxW | stride | halo 8 waves | halo 4 waves | MIOpen | best halo TF/s |\n|---|---|---|---|---|---|---|")
    for c, h, st in SHAPES:
        if only and c not in only:
            continue
        x = torch.randn(args.batch, c, h * st, h * st, device="cuda").bfloat16().contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(args.batch, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(c, c, 3, 3, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        if args.loop:
            for _ in range(args.loop):
                C.wgrad3x3(dy, x, st)
            torch.cuda.synchronize()
            continue
        C.set_wgrad3x3_waves(4)
        t4 = timeit(lambda: C.wgrad3x3(dy, x, st)) if st == 1 else float("nan")
        C.set_wgrad3x3_waves(8)
        th = timeit(lambda: C.wgrad3x3(dy, x, st))
        tm = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
        fl = 2.0 * args.batch * h * h * c * c * 9
        best = th if st != 1 else min(th, t4)
        print(f"| {c} | {h}x{h} | {st} | {th:.3f} | {t4:.3f} | {tm:.3f} | {fl / best / 1e9:.0f} |", flush=True)
    print("done")


if __name__ == "__main__":
    main()
