#!/usr/bin/env python3
"""Cost of the fused epilogues of gemm_xl on the ViT-B/16 linears (batch 256,
50432 tokens): every epilogue mode under the ping-pong (PIPE 7), ring (1) and
persistent (6) main loops, next to the hipBLASLt + separate-pass sequence it
replaces.  HIP events, ms per call."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402


def timeit(fn, iters=10):
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
    C = _native.require("xl epilogue bench")
    T = 50432
    shapes = [("fc1 fwd", 768, 3072), ("fc2 fwd", 3072, 768), ("proj fwd", 768, 768), ("fc2 dgrad", 768, 3072)]
    modes = ["store", "bias", "bias_gelu", "dgelu", "bias_res"]
    print("| shape | pipe | " + " | ".join(modes) + " | lib addmm | lib + gelu / add |")
    print("|---|---|" + "---|" * (len(modes) + 2))
    for name, K, N in shapes:
        x = torch.rand(T, K, device="cuda").bfloat16() * 2 - 1
        w = (torch.rand(N, K, device="cuda").bfloat16() * 2 - 1) * 0.05
        b = torch.rand(N, device="cuda").bfloat16()
        aux = torch.randn(T, N, device="cuda").bfloat16()
        res = torch.randn(T, N, device="cuda").bfloat16()
        kw = {"store": {}, "bias": dict(bias=b), "bias_gelu": dict(bias=b, aux=aux), "dgelu": dict(aux=aux),
              "bias_res": dict(bias=b, residual=res)}
        lib = timeit(lambda: torch.addmm(b, x, w.t()))
        lib2 = timeit(lambda: F.gelu(torch.addmm(b, x, w.t()))) if "fc1" in name else \
            timeit(lambda: res + torch.addmm(b, x, w.t()))
        for pipe in (11, 10, 1):
            C.set_gemm_xl_bn(0, pipe)
            ts = [timeit(lambda: C.gemm_xl(x, w, m, **kw[m])) for m in modes]
            print(f"| {name} | {pipe} | " + " | ".join(f"{t:.3f}" for t in ts) + f" | {lib:.3f} | {lib2:.3f} |",
                  flush=True)
        C.set_gemm_xl_bn(0)
        del x, w, aux, res
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
