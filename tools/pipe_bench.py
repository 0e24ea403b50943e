#!/usr/bin/env python3
"""A/B of the 256 x 256 main loops (csrc/gemm/gemm_xl.hip): PIPE 10 (8-wave
ping-pong, both B halves held in registers, copies issued 4 phases ahead) vs
PIPE 11 (4 waves, 128 x 128 per wave in AGPRs, full-line LDS-DMA), for
the NT kernel (gemm_xl store / conv epilogues / 3x3 implicit GEMM) and the TN
weight-gradient kernel (gemm_tn_xl), on the ViT-B/16 and ResNet-50 shapes
that carry the step time, plus hipBLASLt (torch.matmul) on the plain shapes.

Interleaved rounds in one process (cdna_hip_programming.md rule 24), random
operands (rule 25); prints median / min ms and TF/s per arm and checks the two
arms agree bit for bit (same MFMA order per accumulator).

usage: python tools/pipe_bench.py [--pipes 10,11] [--lib] [--epi] [--rounds 5] [--iters 10] [--only name] [--no-tn]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("pipe bench")

NT_SHAPES = [  # name, M, N, K
    ("vit_qkv_fwd", 50432, 2304, 768),
    ("vit_fc1_fwd", 50432, 3072, 768),
    ("vit_fc2_fwd", 50432, 768, 3072),
    ("vit_fc2_dgrad", 50432, 3072, 768),
    ("r50_l2_1x1", 1605632, 512, 128),
    ("r50_l3_1x1", 401408, 1024, 256),
    ("r50_l4_1x1", 100352, 2048, 512),
    ("r50_l3_dgrad", 401408, 256, 1024),
    ("square_8192", 8192, 8192, 8192),
    ("square_4096", 4096, 4096, 4096),
]
CONV_SHAPES = [  # name, N, C, H (= W), Cout: 3x3 / stride 1 / pad 1 at ResNet-50 batch 2048
    ("r50_l3_3x3", 2048, 256, 14, 256),
    ("r50_l4_3x3", 2048, 512, 7, 512),
    ("r50_l2_3x3", 2048, 128, 28, 128),
]
TN_SHAPES = [  # name, M (reduction), N, K  (ResNet-50 at batch 2048: dW[Cout, Cin] = dy^T x)
    ("vit_fc1_wgrad", 50432, 3072, 768),
    ("vit_qkv_wgrad", 50432, 2304, 768),
    ("r50_l3_wgrad", 401408, 1024, 256),
    ("r50_l2_wgrad", 1605632, 512, 128),
    ("r50_l4_wgrad", 100352, 2048, 512),
    ("r50_l1c1_wgrad", 6422528, 64, 256),
    ("r50_l1c3_wgrad", 6422528, 256, 64),
    ("r50_l2c1_wgrad", 1605632, 128, 512),
    ("r50_l3c1_wgrad", 401408, 256, 1024),
    ("r50_l4c1_wgrad", 100352, 512, 2048),
    ("bs256_l4_wgrad", 12544, 2048, 512),   # batch 256: below the 16k-row threshold
    ("bs256_l4c1_wgrad", 12544, 512, 2048),
    ("bs256_l4c2_wgrad", 12544, 512, 512),
    ("bs256_l3_wgrad", 50176, 1024, 256),
]
WGRAD_SHAPES = [  # name, N, Cin, H_in (= W), Cout, stride: 3x3 / pad 1 weight gradients at batch 2048
    ("r50_l4_3x3wg", 2048, 512, 7, 512, 1),
    ("r50_l4s2_3x3wg", 2048, 512, 14, 512, 2),
    ("r50_l3_3x3wg", 2048, 256, 14, 256, 1),
    ("r50_l3s2_3x3wg", 2048, 256, 28, 256, 2),
]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def ab(name, flops, arms, rounds, iters, exact=None):
    outs = {k: f() for k, f in arms.items()}
    torch.cuda.synchronize()
    ref = next(iter(outs.values()))
    same = {k: (bool(torch.equal(v, ref)) if exact is None or k in exact else True) for k, v in outs.items()}
    rel = {k: float((v.float() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-30))
           for k, v in outs.items()}
    del outs
    times = {k: [] for k in arms}
    for _ in range(rounds):
        for k, f in arms.items():
            f()
            times[k].append(timed(f, iters))
    parts = []
    for k, ts in times.items():
        med = statistics.median(ts)
        parts.append(f"{k} {med:.3f} ms (min {min(ts):.3f}) {flops / med / 1e9:.0f} TF/s"
                     f"{'' if same[k] else ' MISMATCH'}{f' rel {rel[k]:.1e}' if rel[k] else ''}")
    print(f"{name}: " + " | ".join(parts), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pipes", default="10,11")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--no-tn", action="store_true")
    ap.add_argument("--epi", action="store_true", help="also the fused ViT epilogues (bias, bias_gelu, dgelu, bias_res)")
    ap.add_argument("--lib", action="store_true", help="add a hipBLASLt arm on the plain shapes")
    a = ap.parse_args()
    pipes = [int(x) for x in a.pipes.split(",")]
    old_pipe = C.get_gemm_xl_pipe()
    try:
        for name, M, N, K in NT_SHAPES:
            if a.only and a.only not in name:
                continue
            x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            w = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1

            def arm(pipe):
                def f():
                    C.set_gemm_xl_bn(256, pipe, 0)
                    return C.gemm_xl(x, w)
                return f
            arms = {f"pipe{p}": arm(p) for p in pipes}
            if a.lib:
                arms["hipblaslt"] = lambda: x @ w.t()
            ab(name, 2.0 * M * N * K, arms, a.rounds, a.iters, exact={f"pipe{p}" for p in pipes})
            if a.epi and name.startswith("vit"):
                bias = torch.rand(N, device="cuda", dtype=torch.bfloat16) - 0.5
                aux = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
                res = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
                for mode in ("bias", "bias_gelu", "dgelu", "bias_res"):
                    def earm(pipe, mode=mode):
                        def f():
                            C.set_gemm_xl_bn(256, pipe, 0)
                            if mode == "bias":
                                return C.gemm_xl(x, w, mode, bias=bias)
                            if mode == "bias_gelu":
                                return C.gemm_xl(x, w, mode, bias=bias, aux=aux)
                            if mode == "dgelu":
                                return C.gemm_xl(x, w, mode, aux=aux)
                            return C.gemm_xl(x, w, mode, bias=bias, residual=res)
                        return f
                    ab(f"{name}_{mode}", 2.0 * M * N * K, {f"pipe{p}": earm(p) for p in pipes}, a.rounds, a.iters)
                del bias, aux, res
            if name.startswith("r50"):
                def carm(pipe):
                    def f():
                        C.set_gemm_xl_bn(256, pipe, 0)
                        return C.gemm_xl_conv(x, w, "moments")[0]
                    return f
                ab(name + "_moments", 2.0 * M * N * K, {f"pipe{p}": carm(p) for p in pipes}, a.rounds, a.iters)
            del x, w
            torch.cuda.empty_cache()
        for name, nb, cin, h, cout in CONV_SHAPES:
            if a.only and a.only not in name:
                continue
            x = (torch.rand(nb, cin, h, h, device="cuda", dtype=torch.bfloat16) * 2 - 1).contiguous(
                memory_format=torch.channels_last)
            wm = torch.rand(cout, 9 * cin, device="cuda", dtype=torch.bfloat16) * 2 - 1

            def varm(pipe):
                def f():
                    C.set_gemm_xl_bn(256, pipe, 0)
                    return C.conv_xl(x, wm, 3, 3, 1, 1, h, h, "moments")[0]
                return f
            ab(name, 2.0 * nb * h * h * cout * 9 * cin, {f"pipe{p}": varm(p) for p in pipes}, a.rounds, a.iters)
            del x, wm
            torch.cuda.empty_cache()
        C.set_gemm_xl_bn(0, old_pipe, 0)
        if a.no_tn:
            return
        for name, M, N, K in TN_SHAPES:
            if a.only and a.only not in name:
                continue
            dy = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
            xx = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            def tarm(pipe):
                def f():
                    C.set_gemm_xl_bn(0, pipe, 0)
                    return C.gemm_tn_xl(dy, xx, torch.float32)
                return f
            arms = {f"tn_pipe{p}": tarm(p) for p in pipes}
            arms["tn_splitm"] = lambda: C.gemm_tn(dy, xx, torch.float32)
            if a.lib:
                arms["hipblaslt"] = lambda: dy.t().mm(xx)
            ab(name, 2.0 * M * N * K, arms, a.rounds, a.iters, exact=set())
            del dy, xx
            torch.cuda.empty_cache()
        for name, nb, cin, h, cout, st in WGRAD_SHAPES:
            if a.only and a.only not in name:
                continue
            ho = (h - 1) // st + 1
            x = (torch.rand(nb, cin, h, h, device="cuda", dtype=torch.bfloat16) * 2 - 1).contiguous(
                memory_format=torch.channels_last)
            dy = (torch.rand(nb, cout, ho, ho, device="cuda", dtype=torch.bfloat16) * 2 - 1).contiguous(
                memory_format=torch.channels_last)
            dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            w = torch.empty(cout, cin, 3, 3, device="cuda", dtype=torch.bfloat16).contiguous(
                memory_format=torch.channels_last)

            def warm(pipe):
                def f():
                    C.set_gemm_xl_bn(0, pipe, 0)
                    return C.conv_wgrad_xl(dy2, x, 3, 3, st, 1, ho, ho, torch.float32)
                return f
            arms = {f"tn_pipe{p}": warm(p) for p in pipes}
            if a.lib:
                arms["miopen"] = lambda: torch.ops.aten.convolution_backward(
                    dy, x, w, None, [st, st], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1].permute(0, 2, 3, 1).reshape(cout, -1)
            ab(name, 2.0 * nb * ho * ho * cout * 9 * cin, arms, a.rounds, a.iters, exact=set())
            del x, dy, dy2, w
            torch.cuda.empty_cache()
    finally:
        C.set_gemm_xl_bn(0, old_pipe, 0)


if __name__ == "__main__":
    main()
