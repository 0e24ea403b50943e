#!/usr/bin/env python3
"""ViT-B/16 (bs128) per-op device timings: every encoder GEMM in its three
training forms (fwd / dgrad / wgrad) on hipBLASLt (torch) vs our MFMA
kernels, plus attention and the elementwise ops.  HIP-event timing.

  python tools/vit_bench.py [--batch 128] [--tunable]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--tunable", action="store_true")
    ap.add_argument("--ours", action="store_true", help="also time the dmp kernels")
    ap.add_argument("--xl", action="store_true", help="time gemm_xl (fwd/dgrad) and 8192^3 only")
    args = ap.parse_args()
    if args.tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_max_tuning_duration(200)
        os.makedirs("gpurun_out", exist_ok=True)
        torch.cuda.tunable.set_filename("gpurun_out/tunableop_results%d.csv")
    dev, dt = "cuda", torch.bfloat16
    T = args.batch * 197
    D = 768
    shapes = {"qkv": (D, 3 * D), "proj": (D, D), "fc1": (D, 4 * D), "fc2": (4 * D, D)}
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "bgrad": 0.0}
    C = None
    if args.ours:
        from distributed_model_parallel_amd import _C as C  # noqa: N811
    if args.xl:
        return xl_bench(T, D, shapes)
    print(f"{'layer':6s} {'op':6s} {'M':>6s} {'N':>6s} {'K':>6s} {'ms':>8s} {'TF/s':>8s} {'ours ms':>8s} {'TF/s':>8s}")
    for name, (fin, fout) in shapes.items():
        x = torch.randn(T, fin, device=dev, dtype=dt)
        w = torch.randn(fout, fin, device=dev, dtype=dt) * 0.02
        bias = torch.randn(fout, device=dev, dtype=dt)
        dy = torch.randn(T, fout, device=dev, dtype=dt)
        wt = w.t().contiguous()
        cases = [
            ("fwd", T, fout, fin, lambda: F.linear(x, w, bias),
             (lambda: C.gemm_nt(x, w)) if C else None),
            ("dgrad", T, fin, fout, lambda: dy @ w,
             (lambda: C.gemm_nt(dy, wt)) if C else None),
            ("wgrad", fout, fin, T, lambda: dy.t() @ x,
             (lambda: C.gemm_tn(dy, x, torch.bfloat16)) if C else None),
        ]
        for op, m, n, k, fn, ours in cases:
            t = timeit(fn)
            tot[op] += t
            fl = 2.0 * m * n * k
            line = f"{name:6s} {op:6s} {m:6d} {n:6d} {k:6d} {t:8.3f} {fl / t / 1e9:8.1f}"
            if ours is not None:
                try:
                    to = timeit(ours)
                    line += f" {to:8.3f} {fl / to / 1e9:8.1f}"
                except Exception as e:  # noqa: BLE001
                    line += f"  ours failed: {e}"
            print(line, flush=True)
        tb = timeit(lambda: dy.sum(0))
        tot["bgrad"] += tb
        print(f"{name:6s} bgrad  {T:6d} {fout:6d}        {tb:8.3f}  ({T * fout * 2 / tb / 1e6:.0f} GB/s)")
    print("per-layer totals (ms):", {k: round(v, 3) for k, v in tot.items()},
          "x12 =", round(12 * sum(tot.values()), 2))
    B, H, S, Dh = args.batch, 12, 197, 64
    q = torch.randn(B, H, S, Dh, device=dev, dtype=dt, requires_grad=True)
    k = torch.randn_like(q, requires_grad=True)
    v = torch.randn_like(q, requires_grad=True)
    tf = timeit(lambda: F.scaled_dot_product_attention(q, k, v))
    o = F.scaled_dot_product_attention(q, k, v)
    g = torch.randn_like(o)
    tbw = timeit(lambda: torch.autograd.grad(o, (q, k, v), g, retain_graph=True))
    fl = 4.0 * B * H * S * S * Dh
    print(f"sdpa fwd {tf:.3f} ms ({fl / tf / 1e9:.0f} TF/s)  bwd {tbw:.3f} ms ({2.5 * fl / tbw / 1e9:.0f} TF/s)")
    h = torch.randn(T, 4 * D, device=dev, dtype=dt)
    tg = timeit(lambda: F.gelu(h))
    print(f"gelu fwd [{T},{4 * D}] {tg:.3f} ms ({2 * h.numel() * 2 / tg / 1e6:.0f} GB/s)")


def xl_bench(T, D, shapes):
    from distributed_model_parallel_amd import _C as C  # noqa: N811
    dev, dt = "cuda", torch.bfloat16
    print(f"{'case':24s} {'M':>6s} {'N':>6s} {'K':>6s} {'blaslt':>8s} {'TF/s':>7s} | "
          f"{'xl auto':>8s} {'TF/s':>7s} {'bn128':>8s} {'bn256':>8s} {'p0 128':>8s} {'p0 256':>8s}")
    cases = [("square 8192", 8192, 8192, 8192), ("square 4096", 4096, 4096, 4096)]
    for name, (fin, fout) in shapes.items():
        cases.append((f"{name} fwd", T, fout, fin))
        cases.append((f"{name} dgrad", T, fin, fout))
    for name, m, n, k in cases:
        a = torch.rand(m, k, device=dev, dtype=dt) * 2 - 1
        b = torch.rand(n, k, device=dev, dtype=dt) * 2 - 1
        fl = 2.0 * m * n * k
        tb = timeit(lambda: a @ b.t())
        res = []
        for bn, pipe in ((0, 1), (128, 1), (256, 1), (128, 0), (256, 0)):
            C.set_gemm_xl_bn(bn, pipe)
            res.append(timeit(lambda: C.gemm_xl(a, b)))
        C.set_gemm_xl_bn(0)
        print(f"{name:24s} {m:6d} {n:6d} {k:6d} {tb:8.3f} {fl / tb / 1e9:7.1f} | "
              f"{res[0]:8.3f} {fl / res[0] / 1e9:7.1f} {res[1]:8.3f} {res[2]:8.3f} {res[3]:8.3f} {res[4]:8.3f}",
              flush=True)
    # fused epilogues on the fc1 forward shape
    x = torch.randn(T, D, device=dev, dtype=dt)
    w = torch.randn(4 * D, D, device=dev, dtype=dt) * 0.02
    bias = torch.randn(4 * D, device=dev, dtype=dt)
    aux = torch.empty(T, 4 * D, device=dev, dtype=dt)
    t_torch = timeit(lambda: F.gelu(F.linear(x, w, bias)))
    t_xl = timeit(lambda: C.gemm_xl(x, w, "bias_gelu", bias=bias, aux=aux))
    print(f"fc1 fwd+gelu: torch {t_torch:.3f} ms  xl bias_gelu {t_xl:.3f} ms")
    t_plain = timeit(lambda: C.gemm_xl(x, w, "bias", bias=bias))
    print(f"fc1 fwd bias only: xl {t_plain:.3f} ms  torch linear {timeit(lambda: F.linear(x, w, bias)):.3f}")
    # fc2 dgrad + GELU backward
    dy = torch.randn(T, D, device=dev, dtype=dt)
    w2 = torch.randn(D, 4 * D, device=dev, dtype=dt) * 0.02
    w2t = w2.t().contiguous()
    pre = torch.randn(T, 4 * D, device=dev, dtype=dt)
    t_torch = timeit(lambda: torch.ops.aten.gelu_backward(dy @ w2, pre))
    t_xl = timeit(lambda: C.gemm_xl(dy, w2t, "dgelu", aux=pre))
    print(f"fc2 dgrad+gelu_bwd: torch {t_torch:.3f} ms  xl dgelu {t_xl:.3f} ms")
    # residual adds
    h = torch.randn(T, 4 * D, device=dev, dtype=dt)
    b2 = torch.randn(D, device=dev, dtype=dt)
    r = torch.randn(T, D, device=dev, dtype=dt)
    t_torch = timeit(lambda: r + F.linear(h, w2, b2))
    t_xl = timeit(lambda: C.gemm_xl(h, w2, "bias_res", bias=b2, residual=r))
    print(f"fc2 fwd+residual: torch {t_torch:.3f} ms  xl bias_res {t_xl:.3f} ms")
    wp = torch.randn(D, D, device=dev, dtype=dt) * 0.02
    t_torch = timeit(lambda: r + F.linear(x, wp, b2))
    t_xl = timeit(lambda: C.gemm_xl(x, wp, "bias_res", bias=b2, residual=r))
    print(f"proj fwd+residual: torch {t_torch:.3f} ms  xl bias_res {t_xl:.3f} ms")


if __name__ == "__main__":
    main()
