#!/usr/bin/env python3
"""Time the ResNet stem passes at batch N: halo kernels (csrc/conv/stem_halo.hip)
vs the row-tap implicit GEMM (conv_nt / conv_wgrad) vs MIOpen.  HIP events,
median of 20.   python tools/stem_bench.py [--batch 2048]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops.stem import stem_wmat  # noqa: E402
from distributed_model_parallel_amd.utils import miopen_db  # noqa: E402
from tools.wgrad_bench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    miopen_db.seed("use")
    C = _native.require("stem bench")
    n = a.batch
    x = torch.randn(n, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.05).bfloat16().contiguous(memory_format=torch.channels_last)
    wm = stem_wmat(w).contiguous()
    s = C.space_to_depth2(x, 3)
    dy = torch.randn(n * 112 * 112, 64, device="cuda").bfloat16()
    dy4 = dy.view(n, 112, 112, 64).permute(0, 3, 1, 2)
    rows = [
        ("s2d", lambda: C.space_to_depth2(x, 3)),
        ("fwd halo (+moments)", lambda: C.stem_halo_fwd(s, wm, 112, True)),
        ("fwd row-tap GEMM (+moments)", lambda: C.conv_nt(s, wm, 4, 1, 1, 0, 112, 112, mode="moments", kc=64)),
        ("fwd MIOpen", lambda: F.conv2d(x, w, None, 2, 3)),
        ("wgrad halo", lambda: C.stem_halo_wgrad(dy, s, 112, torch.bfloat16)),
        ("wgrad row-tap TN", lambda: C.conv_wgrad(dy, s, 4, 1, 1, 0, 112, 112, torch.bfloat16, kc=64)),
        ("wgrad MIOpen", lambda: torch.ops.aten.convolution_backward(
            dy4, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1, [False, True, False])),
    ]
    fl = 2.0 * n * 112 * 112 * 64 * 147
    print(f"ResNet-50 stem, batch {n}; true FLOP {fl / 1e9:.0f} G")
    print("| pass | ms | TF/s (true FLOP) |\n|---|---|---|")
    for name, fn in rows:
        ms = timeit(fn)
        print(f"| {name} | {ms:.3f} | {fl / ms / 1e9:.0f} |", flush=True)


if __name__ == "__main__":
    main()
