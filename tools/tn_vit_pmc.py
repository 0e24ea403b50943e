#!/usr/bin/env python3
"""PMC driver: the ping-pong TN weight-gradient kernel (gemm_tn_xl) on the
ViT-B/16 fc1 shape (50432 tokens, 3072 x 768 output, 36 tiles x 7 splits) and
on the ResNet-50 layer-3 1x1 shape (401408 rows, 1024 x 256, 4 tiles x 64
splits), a few launches each, so a counter pass can compare where the ViT
shape loses per K step.  Run under `rocprofv3 --pmc ... --kernel-trace`.
With --ablate also times the timing-only ablations of the main loop (1: no
global staging after the prologue, 2: no barriers), HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("tn vit pmc")
for name, M, N, K in (("vit_fc1", 50432, 3072, 768), ("r50_l3", 401408, 1024, 256)):
    a = torch.randn(M, N, device="cuda").bfloat16()
    b = torch.randn(M, K, device="cuda").bfloat16()
    for _ in range(3):
        C.gemm_tn_xl(a, b, torch.bfloat16)
    torch.cuda.synchronize()
    if "--ablate" in sys.argv:
        res = []
        for abl in (0, 1, 2):
            C.set_tn_xl_ablation(abl)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            C.gemm_tn_xl(a, b, torch.bfloat16)
            e0.record()
            for _ in range(10):
                C.gemm_tn_xl(a, b, torch.bfloat16)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            res.append(f"ablation {abl}: {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.0f} TF/s")
        C.set_tn_xl_ablation(0)
        print(name, "; ".join(res), flush=True)
    print(name, "done", flush=True)
    del a, b
