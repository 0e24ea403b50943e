#!/usr/bin/env python3
"""A/B of the two 256 x 256 ping-pong main loops (csrc/gemm/gemm_xl.hip):
PIPE 7 (two tile buffers, 2 units = 32 KB of operands in flight per CU) vs
PIPE 8 (the 10-slot LDS unit ring, 5 units = 80 KB in flight), for the NT
kernel (gemm_xl store / conv epilogues) and the TN weight-gradient kernel
(gemm_tn_xl), on the ViT-B/16 and ResNet-50 shapes that carry the step time.

Interleaved rounds in one process (cdna_hip_programming.md rule 24), random
operands (rule 25); prints median / min ms and TF/s per arm and checks the two
arms agree bit for bit (same MFMA order per accumulator).

usage: python tools/ring_bench.py [--rounds 5] [--iters 10]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("ring bench")

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
]
TN_SHAPES = [  # name, M (reduction), N, K
    ("vit_fc1_wgrad", 50432, 3072, 768),
    ("vit_qkv_wgrad", 50432, 2304, 768),
    ("r50_l3_wgrad", 401408, 1024, 256),
    ("r50_l2_wgrad", 1605632, 512, 128),
    ("r50_l4_wgrad", 100352, 2048, 512),
]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def ab(name, flops, arms, rounds, iters):
    outs = {k: f() for k, f in arms.items()}
    torch.cuda.synchronize()
    ref = next(iter(outs.values()))
    same = {k: bool(torch.equal(v, ref)) for k, v in outs.items()}
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
                     f"{'' if same[k] else ' MISMATCH'}")
    print(f"{name}: " + " | ".join(parts), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    old_pipe, old_ring = C.get_gemm_xl_pipe(), C.get_tn_xl_ring()
    try:
        for name, M, N, K in NT_SHAPES:
            if a.only and a.only not in name:
                continue
            x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            w = torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1

            def arm(pipe):
                def f():
                    C.set_gemm_xl_bn(256, pipe)
                    return C.gemm_xl(x, w)
                return f
            ab(name, 2.0 * M * N * K, {"pipe7": arm(7), "ring8": arm(8)}, a.rounds, a.iters)
            if name.startswith("r50"):
                def carm(pipe):
                    def f():
                        C.set_gemm_xl_bn(256, pipe)
                        return C.gemm_xl_conv(x, w, "moments")[0]
                    return f
                ab(name + "_moments", 2.0 * M * N * K, {"pipe7": carm(7), "ring8": carm(8)}, a.rounds, a.iters)
            del x, w
            torch.cuda.empty_cache()
        C.set_gemm_xl_bn(0, old_pipe)
        for name, M, N, K in TN_SHAPES:
            if a.only and a.only not in name:
                continue
            dy = torch.rand(M, N, device="cuda", dtype=torch.bfloat16) * 2 - 1
            xx = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1

            def tarm(r):
                def f():
                    C.set_tn_xl_ring(r)
                    return C.gemm_tn_xl(dy, xx, torch.float32)
                return f
            ab(name, 2.0 * M * N * K, {"tilebuf": tarm(0), "ring": tarm(1)}, a.rounds, a.iters)
            del dy, xx
            torch.cuda.empty_cache()
    finally:
        C.set_gemm_xl_bn(0, old_pipe)
        C.set_tn_xl_ring(old_ring)


if __name__ == "__main__":
    main()
