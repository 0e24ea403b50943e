#!/usr/bin/env python3
"""BN-fold GEMMs of ResNet-50 at batch 2048 (ops/bn_fold.py), 4-wave NT kernel
vs the 8-wave ping-pong kernel (gemm_xl_conv): the forward
relu(acc * scale + shift + residual) epilogue, and the two-source data
gradient [dz | a] @ Bm^T + ebias with bn2's BN-backward epilogue.  Also the
Gram GEMM a^T a (gemm_tn vs gemm_tn_xl) and the coefficient kernels.
HIP events, ms per call; the HBM column is bytes moved / time."""
import os
import sys

import torch

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
    C = _native.require("bench")
    B = int(os.environ.get("FOLD_BENCH_BATCH", "2048"))
    shapes = [("l1", B * 3136, 64, 256), ("l2", B * 784, 128, 512), ("l3", B * 196, 256, 1024),
              ("l4", B * 49, 512, 2048)]
    print(f"batch {B}")
    print("| layer | M | Cin | Cout | fwd nt | fwd xl | fwd GB/s best | dgrad nt | dgrad xl | gram tn | gram tn_xl | "
          "coef fwd | coef bwd |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|---|")
    for name, M, cin, cout in shapes:
        a = torch.relu(torch.randn(M, cin, device="cuda")).bfloat16()
        w = (torch.randn(cout, cin, device="cuda") * 0.05).bfloat16()
        res = torch.randn(M, cout, device="cuda").bfloat16()
        sc = torch.rand(cout, device="cuda") + 0.5
        sh = torch.randn(cout, device="cuda")
        f_nt = timeit(lambda: C.gemm_nt(a, w, mode="affine", epi_scale=sc, epi_shift=sh, residual=res, relu=True))
        f_xl = timeit(lambda: C.gemm_xl_conv(a, w, "affine", residual=res, scale=sc, shift=sh, relu=True))
        gbs = (2 * M * cout * 2 + M * cin * 2) / min(f_nt, f_xl) / 1e6
        dz = torch.randn(M, cout, device="cuda").bfloat16()
        bm = (torch.randn(cin, cout + cin, device="cuda") * 0.05).bfloat16()
        eb = torch.randn(cin, device="cuda")
        x2 = torch.randn(M, cin, device="cuda").bfloat16()
        mean = torch.zeros(cin, device="cuda")
        inv = torch.ones(cin, device="cuda")
        d_nt = timeit(lambda: C.gemm_nt_bnbwd(dz, bm, None, x2, None, mean, inv, None, None, a2=a, ebias=eb))
        d_xl = timeit(lambda: C.gemm_xl_conv(dz, bm, "bnbwd", bn_x=x2, mean=mean, invstd=inv, a2=a, ebias=eb))
        g_tn = timeit(lambda: C.gemm_tn(a, a, torch.float32))
        g_xl = timeit(lambda: C.gemm_tn_xl(a, a, torch.float32)) if cin >= 256 else float("nan")
        G = C.gemm_tn(a, a, torch.float32)
        ad = a[:4096].double()
        asums = torch.cat([ad.sum(0), (ad * ad).sum(0), ad.new_tensor([float(M)])])
        c_f = timeit(lambda: C.bn_fold_fwd(w, G, asums))
        sums, WG = C.bn_fold_fwd(w, G, asums)
        D = torch.randn(cout, cin, device="cuda")
        sdz = torch.randn(cout, device="cuda", dtype=torch.float64)
        local = C.bn_fold_bwd_sums(D, w, sdz, sh)
        cnt = asums[2 * cin:]
        c_b = timeit(lambda: (C.bn_fold_bwd_sums(D, w, sdz, sh),
                              C.bn_fold_bwd_coef(local, local, cnt, sc, sh, sc, D, WG, asums, w)))
        print(f"| {name} | {M} | {cin} | {cout} | {f_nt:.3f} | {f_xl:.3f} | {gbs:.0f} | {d_nt:.3f} | {d_xl:.3f} | "
              f"{g_tn:.3f} | {g_xl:.3f} | {c_f:.3f} | {c_b:.3f} |", flush=True)
        del a, w, res, dz, bm, x2


if __name__ == "__main__":
    main()
