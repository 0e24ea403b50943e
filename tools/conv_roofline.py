#!/usr/bin/env python3
"""Every ResNet-50 convolution of one training step at batch B, timed per pass
(forward, data gradient, weight gradient) for each backend that can run it --
ours (MFMA NT / TN / implicit-GEMM kernels), MIOpen (F.conv2d /
convolution_backward) and hipBLASLt (torch.mm for 1x1) -- against a roofline
floor max(FLOP / 2.3 PF/s, min HBM bytes / 6 TB/s).  HIP-event timing, no
profiler.  Output: one markdown table, per-pass totals, and the step total of
the per-shape best backend.  Diagnostic for profiles/, not part of the framework.

usage: python tools/conv_roofline.py [--batch 1024]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops.conv_igemm import _wmat  # noqa: E402

PEAK_FLOPS = 2.3e15   # dense bf16 MFMA, realistic clock
PEAK_BYTES = 6.0e12   # sustained HBM3E streaming


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def resnet50_convs():
    """(name, cin, cout, k, stride, H_in, count) of every conv in ResNet-50."""
    out = [("stem", 3, 64, 7, 2, 224, 1)]
    cin = 64
    for li, (planes, blocks, stride, h) in enumerate(((64, 3, 1, 56), (128, 4, 2, 56),
                                                      (256, 6, 2, 28), (512, 3, 2, 14)), 1):
        ho = h // stride
        # first block
        out.append((f"l{li}.b0.conv1", cin, planes, 1, 1, h, 1))
        out.append((f"l{li}.b0.conv2", planes, planes, 3, stride, h, 1))
        out.append((f"l{li}.b0.conv3", planes, planes * 4, 1, 1, ho, 1))
        out.append((f"l{li}.b0.down", cin, planes * 4, 1, stride, h, 1))
        cin = planes * 4
        if blocks > 1:
            out.append((f"l{li}.bN.conv1", cin, planes, 1, 1, ho, blocks - 1))
            out.append((f"l{li}.bN.conv2", planes, planes, 3, 1, ho, blocks - 1))
            out.append((f"l{li}.bN.conv3", planes, planes * 4, 1, 1, ho, blocks - 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--only", default="", help="comma-separated name prefixes (e.g. l4,stem)")
    ap.add_argument("--tn-ab", action="store_true", help="also time weight gradients with narrow TN tiles")
    a = ap.parse_args()
    only = [p for p in a.only.split(",") if p]
    C = _native.require("conv roofline")
    torch.backends.cudnn.benchmark = True
    from distributed_model_parallel_amd.utils import miopen_db
    miopen_db.seed("use")
    B, dev, dt, cl = a.batch, "cuda", torch.bfloat16, torch.channels_last
    rows = []
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}  # best, floor
    print(f"ResNet-50 convolutions, batch {B}, ms per call (HIP events); floor = max(FLOP/{PEAK_FLOPS/1e15:.1f} PF/s, "
          f"bytes/{PEAK_BYTES/1e12:.0f} TB/s)\n")
    print("| conv | x | pass | ours | xl | halo | MIOpen | hipBLASLt | floor | best/floor | TF/s (best) |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for name, cin, cout, k, s, h, cnt in resnet50_convs():
        if only and not any(name.startswith(p) for p in only):
            continue
        pad = k // 2
        ho = (h + 2 * pad - k) // s + 1
        x = torch.randn(B, cin, h, h, device=dev, dtype=dt).contiguous(memory_format=cl)
        w = (torch.randn(cout, cin, k, k, device=dev, dtype=dt) * 0.05).contiguous(memory_format=cl)
        dy = torch.randn(B, cout, ho, ho, device=dev, dtype=dt).contiguous(memory_format=cl)
        flops = 2.0 * B * ho * ho * cout * cin * k * k
        bx, by, bw = x.numel() * 2, dy.numel() * 2, w.numel() * 2
        floors = {"fwd": max(flops / PEAK_FLOPS, (bx + by + bw) / PEAK_BYTES) * 1e3,
                  "dgrad": max(flops / PEAK_FLOPS, (bx + by + bw) / PEAK_BYTES) * 1e3,
                  "wgrad": max(flops / PEAK_FLOPS, (bx + by + bw) / PEAK_BYTES) * 1e3}
        res = {p: {} for p in floors}
        geom = [] if s == 1 else [s, ho, ho, h, h]
        x2 = x.permute(0, 2, 3, 1).reshape(-1, cin)
        dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
        # MIOpen (every conv)
        res["fwd"]["miopen"] = timeit(lambda: F.conv2d(x, w, None, s, pad))
        res["dgrad"]["miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1, (True, False, False)))
        res["wgrad"]["miopen"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, (s, s), (pad, pad), (1, 1), False, (0, 0), 1, (False, True, False)))
        if name == "stem":
            from distributed_model_parallel_amd.ops.stem import stem_wmat
            wm = stem_wmat(w)
            res["fwd"]["ours"] = timeit(lambda: C.conv_nt(C.space_to_depth2(x, 3), wm, 4, 1, 1, 0, ho, ho,
                                                          mode="moments", kc=64))
            s2d = C.space_to_depth2(x, 3)
            res["wgrad"]["ours"] = timeit(lambda: C.conv_wgrad(dy2, s2d, 4, 1, 1, 0, ho, ho, dt, kc=64))
        elif k == 1:
            w2 = w.view(cout, cin)
            wt = w2.t().contiguous()
            res["fwd"]["ours"] = timeit(lambda: C.gemm_nt(x2, w2, mode="moments", a_map=geom))
            res["dgrad"]["ours"] = timeit(lambda: C.gemm_nt(dy2, wt, c_map=geom))
            res["wgrad"]["ours"] = timeit(lambda: C.gemm_tn(dy2, x2, dt, b_map=geom))
            if hasattr(C, "gemm_tn_xl") and s == 1 and cout >= 128 and cin >= 256:
                res["wgrad"]["xl"] = timeit(lambda: C.gemm_tn_xl(dy2, x2, dt))
            if s == 1:
                res["fwd"]["blaslt"] = timeit(lambda: x2 @ w2.t())
                res["dgrad"]["blaslt"] = timeit(lambda: dy2 @ w2)
                res["wgrad"]["blaslt"] = timeit(lambda: dy2.t() @ x2)
        elif cin % 64 == 0:
            res["fwd"]["ours"] = timeit(lambda: C.conv_nt(x, _wmat(w), k, k, s, pad, ho, ho, mode="moments"))
            wtr = w.permute(1, 2, 3, 0).reshape(cin, -1).contiguous()
            res["dgrad"]["ours"] = timeit(lambda: C.conv_nt(dy, wtr, k, k, s, pad, h, h, transposed=True))
            res["wgrad"]["ours"] = timeit(lambda: C.conv_wgrad(dy2, x, k, k, s, pad, ho, ho, dt))
            if hasattr(C, "wgrad3x3") and k == 3 and cin == cout and C.wgrad3x3_supported(cin, ho, ho, s):
                res["wgrad"]["halo"] = timeit(lambda: C.wgrad3x3(dy, x, s))
            if hasattr(C, "conv_wgrad_xl") and cin % 256 == 0:
                res["wgrad"]["xl"] = timeit(lambda: C.conv_wgrad_xl(dy2, x, k, k, s, pad, ho, ho, dt))
            if hasattr(C, "conv_xl") and k > 1:  # 256x256 ping-pong implicit GEMM
                res["fwd"]["xl"] = timeit(lambda: C.conv_xl(x, _wmat(w), k, k, s, pad, ho, ho, "moments"))
                if s == 1:
                    wfl = w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, -1).contiguous()
                    res["dgrad"]["xl"] = timeit(lambda: C.conv_xl(dy, wfl, k, k, 1, pad, h, h, "store"))
                elif k == 3 and s == 2 and cin % 256 == 0 and hasattr(C, "conv_xl_dgrad_s2"):
                    from distributed_model_parallel_amd.ops.conv_igemm import _phase_weights
                    wph = _phase_weights(w)
                    res["dgrad"]["xl"] = timeit(lambda: C.conv_xl_dgrad_s2(dy, wph, h, h))
            from distributed_model_parallel_amd.ops.conv_igemm import _halo_conv, _halo_dgrad_s2_ok, _halo_kind
            hk = _halo_kind(cin, cout, k, k, s, pad, h, h)
            if _halo_dgrad_s2_ok(cin, cout, k, k, s, pad, h, h):
                wt_ = w.permute(1, 2, 3, 0).reshape(cin, -1).contiguous()
                res["dgrad"]["halo"] = timeit(lambda: C.conv3x3_c128_dgrad_s2(dy, wt_))
            if hk:  # halo-tiled 3x3 (layers 1-2): forward with moments, dgrad over flipped weights
                wfl = w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, -1).contiguous()
                res["fwd"]["halo"] = timeit(lambda: _halo_conv(C, hk)(x, _wmat(w).contiguous(), True))
                res["dgrad"]["halo"] = timeit(lambda: _halo_conv(C, hk)(dy, wfl, False))
        if a.tn_ab and "ours" in res["wgrad"] and name != "stem":
            # A/B of the 128 x 256 TN tile: the narrow-tile time under its own column
            C.set_tn_wide(False)
            if k == 1:
                res["wgrad"]["narrow"] = timeit(lambda: C.gemm_tn(dy2, x2, dt, b_map=geom))
            else:
                res["wgrad"]["narrow"] = timeit(lambda: C.conv_wgrad(dy2, x, k, k, s, pad, ho, ho, dt))
            C.set_tn_wide(True)
            print(f"  {name} wgrad: wide-enabled {res['wgrad']['ours']:.3f} narrow {res['wgrad']['narrow']:.3f}")
        for p in ("fwd", "dgrad", "wgrad"):
            if name == "stem" and p == "dgrad":
                continue  # the input image needs no gradient
            r = res[p]
            best = min(r.values())
            tot[p][0] += best * cnt
            tot[p][1] += floors[p] * cnt
            f = lambda k_: f"{r[k_]:.3f}" if k_ in r else "-"  # noqa: E731
            print(f"| {name} | {cnt} | {p} | {f('ours')} | {f('xl')} | {f('halo')} | {f('miopen')} | {f('blaslt')} | "
                  f"{floors[p]:.3f} | "
                  f"{best / floors[p]:.2f} | {flops / best / 1e9:.0f} |")
        del x, w, dy, x2, dy2
        torch.cuda.empty_cache()
    print("\n| pass | best backend per shape, ms/step | floor ms/step |")
    print("|---|---|---|")
    for p, (b, fl) in tot.items():
        print(f"| {p} | {b:.2f} | {fl:.2f} |")
    print(f"| all | {sum(v[0] for v in tot.values()):.2f} | {sum(v[1] for v in tot.values()):.2f} |")


if __name__ == "__main__":
    main()
