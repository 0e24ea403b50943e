#!/usr/bin/env python3
"""PMC driver: the ping-pong TN weight-gradient kernel (gemm_tn_xl) on the
ViT-B/16 fc1 shape (50432 tokens, 3072 x 768 output, 36 tiles x 7 splits) and
on the ResNet-50 layer-3 1x1 shape (401408 rows, 1024 x 256, 4 tiles x 64
splits), a few launches each, so a counter pass can compare where the ViT
shape loses per K step.  Run under `rocprofv3 --pmc ... --kernel-trace`."""
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
    print(name, "done", flush=True)
    del a, b
