#!/usr/bin/env python3
"""Time the halo-tiled 3x3 convs against MIOpen (find mode, seeded db) and the
implicit-GEMM conv_nt at batch N (default 1024): forward (+ BN moments for
ours), data gradient.  --c 64: ResNet-50 layer 1's conv2 (csrc/conv/
conv3x3_halo.hip, 56x56); --c 128: layer 2's (csrc/conv/conv3x3_c128.hip,
28x28).  HIP events, median of 20 after 5 warm-up calls.

  python tools/halo_bench.py [--batch 1024] [--c 64|128]
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
    ap.add_argument("--c", type=int, default=64, choices=(64, 128))
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    miopen_db.seed("use")
    C = _native.require("halo_bench")
    c = args.c
    n, h = args.batch, (56 if c == 64 else 28)
    halo = C.conv3x3_c64 if c == 64 else C.conv3x3_c128
    x = torch.randn(n, c, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") / (3 * c ** 0.5)).bfloat16().contiguous(
        memory_format=torch.channels_last)
    wm = conv_igemm._wmat(w).contiguous()
    wfl = w.flip(2, 3).permute(1, 2, 3, 0).reshape(c, -1).contiguous()
    floor = 2 * x.numel() * 2 / 6e12 * 1e3
    flop = 2.0 * x.numel() * c * 9
    rows = [
        ("fwd halo (+moments)", lambda: halo(x, wm, True)),
        ("fwd halo (store)", lambda: halo(x, wm, False)),
        ("fwd conv_nt (+moments)", lambda: C.conv_nt(x, wm, 3, 3, 1, 1, h, h, mode="moments")),
        ("fwd MIOpen", lambda: F.conv2d(x, w, None, 1, 1)),
        ("dgrad halo", lambda: halo(x, wfl, False)),
        ("dgrad MIOpen", lambda: torch.ops.aten.convolution_backward(
            x, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
    ]
    print(f"ResNet-50 3x3 {c}->{c} on {h}x{h}, batch {n}; HBM floor {floor:.3f} ms")
    print("| pass | ms | TB/s (x + y) | TF/s |\n|---|---|---|---|")
    for name, fn in rows:
        ms = timeit(fn)
        print(f"| {name} | {ms:.3f} | {2 * x.numel() * 2 / ms / 1e9:.2f} | {flop / ms / 1e9:.0f} |", flush=True)


if __name__ == "__main__":
    main()
