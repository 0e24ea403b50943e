#!/usr/bin/env python3
"""ViT-B/16 attention (B=128, S=197, H=12, Dh=64): packed-qkv HIP kernels vs
the SDPA path including its layout copies.  HIP-event timing."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.ops import attention as A  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
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


def sdpa_path(qkv, heads):
    b, s, d3 = qkv.shape
    d = d3 // 3
    q, k, v = qkv.view(b, s, 3, heads, d // heads).permute(2, 0, 3, 1, 4).unbind(0)
    o = F.scaled_dot_product_attention(q, k, v)
    return o.transpose(1, 2).reshape(b, s, d)


def main():
    B, S, H = int(os.environ.get("B", 128)), 197, 12
    # VARIANT="f,b" ITERS=n: only that variant, n forward + backward passes (profiling)
    only = os.environ.get("VARIANT")
    qkv = torch.randn(B, S, 3 * H * 64, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    go = torch.randn(B, S, H * 64, device="cuda", dtype=torch.bfloat16)
    from distributed_model_parallel_amd import _native
    C = _native.require("attn bench")

    def variant(v, vb):
        def f():
            C.set_attention_variant(v, vb)
            return A.self_attention_packed(qkv, H)
        return f
    if only:
        f = variant(*(int(x) for x in only.split(",")))
        for _ in range(int(os.environ.get("ITERS", 3))):
            torch.autograd.grad(f(), qkv, go)
        torch.cuda.synchronize()
        print("done", only)
        return
    for name, fn in (("sdpa+copies", lambda: sdpa_path(qkv, H)), ("hip per-head", variant(0, 0)),
                     ("hip persistent", variant(1, 1)), ("hip 8-wave fwd", variant(2, 1)),
                     ("hip pers fwd + per-head bwd", variant(1, 0)), ("hip 2-tile fwd", variant(3, 0))):
        tf = timeit(lambda: fn())
        o = fn()
        tb = timeit(lambda: torch.autograd.grad(o, qkv, go, retain_graph=True))
        fl = 4.0 * B * H * S * S * 64
        print(f"{name:12s} fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF/s)  bwd {tb:.3f} ms ({2.5 * fl / tb / 1e9:.0f} TF/s)"
              f"  total {tf + tb:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
