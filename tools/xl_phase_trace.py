#!/usr/bin/env python3
"""Where a ping-pong GEMM tile's time goes (gemm_xl.hip PIPE 7,
set_gemm_xl_trace): per block, thread 0 records the realtime clock (10 ns) at
entry, when the first K tile's operands have landed, after the main loop and
after the epilogue, plus the HW_ID / XCC_ID registers that name its CU.  This
tool runs ResNet-50 batch-2048 GEMMs with tracing on and reports, per GEMM:
the median prologue / main loop / epilogue of a tile, the gap between one
tile's end and the next tile's start on the same CU, and how busy the CUs
were over the kernel's span.

usage: python tools/xl_phase_trace.py [--batch 2048]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_model_parallel_amd import _native  # noqa: E402


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def analyse(buf: torch.Tensor, blocks: int):
    t = buf[: blocks * 8].view(blocks, 8).cpu()
    ok = (t[:, 0] > 0) & (t[:, 3] >= t[:, 0])
    t = t[ok]
    t0 = int(t[:, 0].min())
    s, l, m, e = ((t[:, k] - t0).double() * 0.01 for k in range(4))  # us
    hw, xcc = t[:, 4], t[:, 5]
    cu = (xcc & 0xF) * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    gaps = []
    per_cu = {}
    for i in range(t.shape[0]):
        per_cu.setdefault(int(cu[i]), []).append((float(s[i]), float(e[i])))
    for v in per_cu.values():
        v.sort()
        gaps += [b[0] - a[1] for a, b in zip(v, v[1:])]
    span = float(e.max())
    busy = sum(b - a for v in per_cu.values() for a, b in v)
    return {"tiles": int(t.shape[0]), "cus": len(per_cu), "span_us": span,
            "prologue_us": med((l - s).tolist()), "main_us": med((m - l).tolist()),
            "epilogue_us": med((e - m).tolist()), "tile_us": med((e - s).tolist()),
            "gap_us": med(gaps), "busy": busy / (span * len(per_cu)) if span > 0 else 0.0,
            "first_round_start_spread_us": float(s.sort().values[min(len(s) - 1, 255)])}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    a = ap.parse_args()
    C = _native.require("xl_phase_trace")
    dev, bf = "cuda", torch.bfloat16
    cases = []
    for name, hw, w in (("l2", 28 * 28, 128), ("l3", 14 * 14, 256), ("l4", 7 * 7, 512)):
        M = a.batch * hw
        x = torch.randn(M, w, device=dev, dtype=bf)
        B = (torch.randn(4 * w, w, device=dev) * 0.05).to(bf)
        R = torch.randn(M, 4 * w, device=dev, dtype=bf)
        sc = torch.rand(4 * w, device=dev) + 0.5
        sh = torch.randn(4 * w, device=dev) * 0.1
        nb = (M + 255) // 256 * (4 * w // 256)
        cases.append((f"{name} fwd moments {M}x{4 * w}x{w}", nb, lambda x=x, B=B: C.gemm_xl_conv(x, B, "moments")))
        cases.append((f"{name} fwd affine+res+relu {M}x{4 * w}x{w}", nb,
                      lambda x=x, B=B, R=R, sc=sc, sh=sh: C.gemm_xl_conv(x, B, "affine", residual=R, scale=sc,
                                                                        shift=sh, relu=True)))
    xs = torch.randn(a.batch, 256, 14, 14, device=dev).to(bf).contiguous(memory_format=torch.channels_last)
    ws = (torch.randn(256, 9 * 256, device=dev) * 0.03).to(bf)
    M3 = a.batch * 196
    C.set_gemm_xl_bm(-1)
    cases.append((f"l3 3x3 conv_xl moments {M3}x256x2304", (M3 + 255) // 256,
                  lambda: C.conv_xl(xs, ws, 3, 3, 1, 1, 14, 14, "moments")))
    print("| GEMM | tiles | CUs | span us | tile us | prologue us | main loop us | epilogue us | gap us | CU busy |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for name, nb, fn in cases:
        for _ in range(2):
            fn()
        buf = torch.zeros(nb * 8 + 64, dtype=torch.long, device=dev)
        torch.cuda.synchronize()
        C.set_gemm_xl_trace(buf)
        fn()
        torch.cuda.synchronize()
        C.set_gemm_xl_trace(None)
        r = analyse(buf, nb)
        print(f"| {name} | {r['tiles']} | {r['cus']} | {r['span_us']:.1f} | {r['tile_us']:.2f} | "
              f"{r['prologue_us']:.2f} | {r['main_us']:.2f} | {r['epilogue_us']:.2f} | {r['gap_us']:.2f} | "
              f"{100 * r['busy']:.1f} % |", flush=True)
    C.set_gemm_xl_bm(0)
    return 0


if __name__ == "__main__":
    sys.exit(main())
