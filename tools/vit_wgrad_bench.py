#!/usr/bin/env python3
"""ViT-B/16 linear weight gradients dW = dy^T x (batch 256: 50432 token rows)
on hipBLASLt (dy.t() @ x) vs our ping-pong TN kernel (gemm_tn_xl, split-M
with a final reduce) vs the 4-wave TN kernel (gemm_tn).  HIP events, ms per
call and TF/s; max |err| of ours against hipBLASLt relative to its max."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, iters=20):
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
    C = _native.require("vit wgrad bench")
    T = int(os.environ.get("VIT_TOKENS", str(256 * 197)))
    shapes = [("qkv", 768, 2304), ("proj", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)]
    print(f"tokens {T}")
    print("| layer | in | out | hipBLASLt ms | tn_xl ms | tn ms | TF/s lib | TF/s tn_xl | rel err |")
    print("|---|---|---|---|---|---|---|---|---|")
    for name, fin, fout in shapes:
        x = torch.randn(T, fin, device="cuda").bfloat16()
        dy = (torch.randn(T, fout, device="cuda") * 0.1).bfloat16()
        lib = timeit(lambda: dy.t() @ x)
        xl = timeit(lambda: C.gemm_tn_xl(dy, x, torch.bfloat16))
        tn = timeit(lambda: C.gemm_tn(dy, x, torch.bfloat16))
        ref = (dy.t() @ x).float()
        sweep = []
        for r in (2, 3, 4):  # split count: r rounds of 256 blocks (0 = the default rule)
            C.set_tn_xl_rounds(r)
            sweep.append(f"r{r} {timeit(lambda: C.gemm_tn_xl(dy, x, torch.bfloat16)):.3f}")
        C.set_tn_xl_rounds(0)
        print("   tn_xl rounds sweep:", ", ".join(sweep))
        err = ((C.gemm_tn_xl(dy, x, torch.bfloat16).float() - ref).abs().max() / ref.abs().max()).item()
        fl = 2.0 * T * fin * fout
        print(f"| {name} | {fin} | {fout} | {lib:.3f} | {xl:.3f} | {tn:.3f} | {fl / lib / 1e9:.0f} | "
              f"{fl / xl / 1e9:.0f} | {err:.1e} |", flush=True)
        del x, dy, ref


if __name__ == "__main__":
    main()
