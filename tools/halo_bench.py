#!/usr/bin/env python3
"""Time the halo-tiled 3x3 64->64 conv (csrc/conv/conv3x3_halo.hip) against
MIOpen (find mode, seeded db) and the implicit-GEMM conv_nt on ResNet-50
layer 1's conv2 at batch N (default 1024): forward (+ BN moments for ours),
data gradient.  HIP events, median of 20 after 5 warm-up calls.

  python tools/halo_bench.py [--batch 1024]
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops import conv_igemm  # noqa: E402
from distributed_model_parallel_amd.utils import miopen_db  # noqa: E402


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
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    miopen_db.seed("use")
    C = _native.require("halo_bench")
    n, h = args.batch, 56
    x = torch.randn(n, 64, h, 56, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, device="cuda") / 24).bfloat16().contiguous(memory_format=torch.channels_last)
    wm = conv_igemm._wmat(w).contiguous()
    wfl = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, -1).contiguous()
    floor = 2 * x.numel() * 2 / 6e12 * 1e3
    rows = [
        ("fwd halo (+moments)", lambda: C.conv3x3_c64(x, wm, True)),
        ("fwd halo (store)", lambda: C.conv3x3_c64(x, wm, False)),
        ("fwd conv_nt (+moments)", lambda: C.conv_nt(x, wm, 3, 3, 1, 1, h, 56, mode="moments")),
        ("fwd MIOpen", lambda: F.conv2d(x, w, None, 1, 1)),
        ("dgrad halo", lambda: C.conv3x3_c64(x, wfl, False)),
        ("dgrad MIOpen", lambda: torch.ops.aten.convolution_backward(
            x, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
    ]
    print(f"ResNet-50 l1 conv2 (3x3, 64->64, 56x56), batch {n}; HBM floor {floor:.3f} ms")
    print("| pass | ms | TB/s (x + y) |\n|---|---|---|")
    for name, fn in rows:
        ms = timeit(fn)
        print(f"| {name} | {ms:.3f} | {2 * x.numel() * 2 / ms / 1e9:.2f} |", flush=True)


if __name__ == "__main__":
    main()
