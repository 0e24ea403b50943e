#!/usr/bin/env python3
"""Tiny driver for PMC passes: the ping-pong TN weight-gradient kernel and the
ping-pong NT kernel on equal-FLOP problems (ResNet-50 layer-3 1x1 wgrad
shape), a few launches each.  Run under rocprofv3 --pmc."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402

C = _native.require("tn pmc")
M, N, K = 200704, 256, 1024
a = torch.randn(M, N, device="cuda").bfloat16()
b = torch.randn(M, K, device="cuda").bfloat16()
x = torch.randn(M // 64, M // 64 * 0 + 4096, device="cuda").bfloat16()  # NT: [3136, 4096] @ [4096, ...]
A2 = torch.randn(4096, 200704 // 8, device="cuda").bfloat16()
B2 = torch.randn(256 * 4, 200704 // 8, device="cuda").bfloat16()
for _ in range(3):
    C.gemm_tn_xl(a, b, torch.float32)
    C.gemm_tn(a, b, torch.float32)
    C.gemm_xl(A2, B2)
torch.cuda.synchronize()
print("done")
