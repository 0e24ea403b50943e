"""gemm_x2_kernel (two 256x128 blocks per CU, register epilogue) against the
one-block-per-CU gemm_xl ring kernel on every conv epilogue it serves:
moments, add, affine (scale / shift / residual / relu / two-source A) and the
fused BN backward (mask from x or y, full and compact strided residual).
Same operands, same K order, same rounding points -> the stored tensors agree
to bf16 rounding and the fp32/fp64 column sums to summation order."""
import pytest
import torch

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture
def C():
    c = _native.require("gemm_x2 tests")
    old = c.get_gemm_xl_x2()
    yield c
    c.set_gemm_xl_x2(old)


def both(C, fn):
    C.set_gemm_xl_x2(0)
    ref = fn()
    C.set_gemm_xl_x2(2)
    out = fn()
    torch.cuda.synchronize()
    return ref, out


def close(a, b, atol=2e-2, rtol=1e-2):
    if isinstance(a, (list, tuple)):
        for x, y in zip(a, b):
            if x is not None:
                close(x, y, atol, rtol)
        return
    if a.dtype == torch.bfloat16:
        torch.testing.assert_close(b.float(), a.float(), atol=atol, rtol=rtol)
    else:
        torch.testing.assert_close(b.double(), a.double(), atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (3001, 512, 128), (50176, 1024, 256), (700, 128, 192),
                                   (6272, 2048, 512), (1000, 384, 1024)])
def test_x2_moments(C, M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    (c0, m0), (c1, m1) = both(C, lambda: C.gemm_xl_conv(a, b, "moments"))
    close(c0, c1)
    cd = c1.double()
    torch.testing.assert_close(m1[:N], cd.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(m1[N:2 * N], (cd * cd).sum(0), atol=1e-2, rtol=1e-4)
    assert m1[2 * N].item() == M
    close(m0, m1)


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (1999, 512, 256)])
def test_x2_add(C, M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    (c0, _), (c1, _) = both(C, lambda: C.gemm_xl_conv(a, b, "add", residual=r))
    close(c0, c1)
    torch.testing.assert_close(c1.float(), (a.float() @ b.float().t() + r.float()), atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("scale,residual,relu", [(True, False, True), (False, True, True), (True, True, False)])
@pytest.mark.parametrize("M,N,K", [(12544, 256, 64), (777, 1024, 512)])
def test_x2_affine(C, M, N, K, scale, residual, relu):
    torch.manual_seed(2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    sc = torch.rand(N, device=DEV) + 0.5 if scale else None
    sh = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).bfloat16() if residual else None
    (c0, _), (c1, _) = both(C, lambda: C.gemm_xl_conv(a, b, "affine", scale=sc, shift=sh, residual=r, relu=relu))
    close(c0, c1)
    ref = a.float() @ b.float().t()
    if sc is not None:
        ref = ref * sc
    ref = ref + sh
    if r is not None:
        ref = ref + r.float()
    if relu:
        ref = torch.relu(ref)
    torch.testing.assert_close(c1.float(), ref, atol=6e-2, rtol=2e-2)


def test_x2_affine_two_source(C):
    """Folded downsample block: [a | x[::2, ::2]] @ [W3 | Wd]^T, A2 read through
    the strided map."""
    torch.manual_seed(3)
    n, hi, cx, cin, cout, s = 4, 14, 256, 128, 512, 2
    ho = hi // s
    geom = [s, ho, ho, hi, hi]
    x2 = torch.relu(torch.randn(n * hi * hi, cx, device=DEV)).bfloat16()
    xs = x2.view(n, hi, hi, cx)[:, ::s, ::s].reshape(-1, cx)
    a = torch.relu(torch.randn(n * ho * ho, cin, device=DEV)).bfloat16()
    Bf = (torch.randn(cout, cin + cx, device=DEV) * 0.05).bfloat16()
    sh = torch.randn(cout, device=DEV)
    (c0, _), (c1, _) = both(C, lambda: C.gemm_xl_conv(a, Bf, "affine", shift=sh, relu=True, a2=x2, a2_map=geom))
    close(c0, c1)
    ref = torch.relu(torch.cat([a, xs], 1).float() @ Bf.float().t() + sh)
    torch.testing.assert_close(c1.float(), ref, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("mask_from_y", [False, True])
@pytest.mark.parametrize("with_res", [False, True])
@pytest.mark.parametrize("M,N,K", [(5000, 256, 128), (25088, 1024, 256)])
def test_x2_bnbwd(C, M, N, K, mask_from_y, with_res):
    torch.manual_seed(4)
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    x = torch.randn(M, N, device=DEV).bfloat16()
    mean = x.float().mean(0)
    inv = torch.rand(N, device=DEV) + 0.5
    bw = torch.rand(N, device=DEV) + 0.5
    bb = torch.randn(N, device=DEV) * 0.5
    res = torch.randn(M, N, device=DEV).bfloat16() if with_res else None
    y = torch.relu(x.float() * inv * bw + bb - mean * inv * bw).bfloat16() if mask_from_y else None
    i_, w_, b_ = (None, None, None) if mask_from_y else (inv, bw, bb)
    r0, r1 = both(C, lambda: C.gemm_xl_conv(dy, wt, "bnbwd", residual=res, bn_x=x, bn_y=y, mean=mean,
                                            invstd=i_, weight=w_, bias=b_))
    close(r0[0], r1[0])
    torch.testing.assert_close(r1[1].double(), r0[1].double(), atol=5e-2, rtol=1e-3)


def test_x2_bnbwd_compact_residual(C):
    """A stride-2 compact residual (res_map) equals the zero-expanded full one."""
    torch.manual_seed(5)
    n, h, w, s, N, K = 3, 10, 9, 2, 256, 128
    ho, wo = (h + 1) // 2, (w + 1) // 2
    M = n * h * w
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    x = torch.randn(M, N, device=DEV).bfloat16()
    mean = x.float().mean(0)
    inv = torch.rand(N, device=DEV) + 0.5
    bb = torch.randn(N, device=DEV) * 0.5
    comp = torch.randn(n * ho * wo, N, device=DEV).bfloat16()
    full = torch.zeros(n, h, w, N, device=DEV).bfloat16()
    full[:, ::s, ::s] = comp.view(n, ho, wo, N)
    full = full.view(M, N)
    C.set_gemm_xl_x2(2)
    a = C.gemm_xl_conv(dy, wt, "bnbwd", residual=comp, bn_x=x, mean=mean, invstd=inv, bias=bb, res_map=[s, ho, wo, h, w])
    b = C.gemm_xl_conv(dy, wt, "bnbwd", residual=full, bn_x=x, mean=mean, invstd=inv, bias=bb)
    torch.testing.assert_close(a[0], b[0])
    torch.testing.assert_close(a[1], b[1], atol=1e-6, rtol=1e-9)


def test_x2_falls_back_when_n_not_multiple_of_128(C):
    torch.manual_seed(6)
    a = torch.randn(1024, 64, device=DEV).bfloat16()
    b = (torch.randn(192, 64, device=DEV) * 0.1).bfloat16()
    (c0, m0), (c1, m1) = both(C, lambda: C.gemm_xl_conv(a, b, "moments"))
    torch.testing.assert_close(c0, c1)
    torch.testing.assert_close(m0, m1)


@pytest.mark.parametrize("w,rows", [(128, 4096 + 77), (256, 2048 + 33)])
def test_fold_dgrad_bnbwd_xl_matches_nt(C, w, rows):
    """The folded bottleneck data gradient da = [dz | a] @ Bb^T + ebias with the
    producer BN's backward in the epilogue, as ops/bn_fold._FoldDgrad routes it
    from round 4 (N = 128 / 256 on gemm_xl_conv: x2 / ping-pong kernel) against
    the NT conv GEMM it used before (same operands, same reduction)."""
    torch.manual_seed(5)
    dz = torch.randn(rows, 4 * w, device=DEV).bfloat16()
    a = torch.randn(rows, w, device=DEV).bfloat16()
    Bb = (torch.randn(w, 5 * w, device=DEV) * 0.05).bfloat16()
    eb = torch.randn(w, device=DEV) * 0.1
    x = torch.randn(rows, w, device=DEV).bfloat16()
    mean = torch.randn(w, device=DEV) * 0.1
    inv = torch.rand(w, device=DEV) + 0.5
    bw = torch.rand(w, device=DEV) + 0.5
    bb = torch.randn(w, device=DEV) * 0.1
    ref, rs = C.gemm_nt_bnbwd(dz, Bb, None, x, None, mean, inv, bw, bb, a2=a, ebias=eb)
    out, os_ = C.gemm_xl_conv(dz, Bb, "bnbwd", bn_x=x, mean=mean, invstd=inv, weight=bw, bias=bb, a2=a, ebias=eb)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), ref.float(), atol=3e-2, rtol=1e-2)
    tol = 2e-2 * rows ** 0.5
    torch.testing.assert_close(os_[: 2 * w], rs[: 2 * w], atol=tol, rtol=1e-2)
