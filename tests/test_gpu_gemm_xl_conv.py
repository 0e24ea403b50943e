"""gemm_xl conv epilogues (moments / add / bnbwd) on the glds-ring kernel must
agree with the 4-wave NT kernel's (gemm_nt / gemm_nt_bnbwd) -- same math,
same rounding points -- and with fp64 sums of what they store."""
import pytest
import torch

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def C():
    return _native.require("gemm_xl_conv tests")


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (3001, 512, 128), (50176, 1024, 256), (700, 128, 192)])
def test_xl_moments_matches_nt(M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    c, mom = C().gemm_xl_conv(a, b, "moments")
    c0, _ = C().gemm_nt(a, b)
    torch.testing.assert_close(c.float(), c0.float(), atol=2e-2, rtol=1e-2)
    cd = c.double()
    torch.testing.assert_close(mom[:N], cd.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(mom[N:2 * N], (cd * cd).sum(0), atol=1e-2, rtol=1e-4)
    assert mom[2 * N].item() == M


@pytest.mark.parametrize("M,N,K", [(4096, 256, 64), (1999, 512, 256)])
def test_xl_add_matches_nt(M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    c, _ = C().gemm_xl_conv(a, b, "add", residual=r)
    c0, _ = C().gemm_nt(a, b, mode="add", residual=r)
    torch.testing.assert_close(c.float(), c0.float(), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("mask_from_y", [False, True])
@pytest.mark.parametrize("with_res", [False, True])
def test_xl_bnbwd_matches_nt(mask_from_y, with_res):
    torch.manual_seed(2)
    M, N, K = 5000, 256, 128
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
    dz, sums = C().gemm_xl_conv(dy, wt, "bnbwd", residual=res, bn_x=x, bn_y=y, mean=mean, invstd=i_,
                                weight=w_, bias=b_)
    dz0, sums0 = C().gemm_nt_bnbwd(dy, wt, res, x, y, mean, i_, w_, b_)
    torch.testing.assert_close(dz.float(), dz0.float(), atol=2e-2, rtol=1e-2)
    dzd = dz.double()
    torch.testing.assert_close(sums[:N], dzd.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(sums[N:2 * N], (dzd * (x.double() - mean.double())).sum(0), atol=1e-2, rtol=1e-4)


@pytest.mark.parametrize("pipe", [10, 11])
@pytest.mark.parametrize("mode", ["moments", "bnbwd"])
def test_xl_conv_pingpong_schedule(mode, pipe):
    """The 256 x 256 main loops (PIPE 10: 8-wave ping-pong, PIPE 11: 4 waves)
    under the conv epilogues equal the half-step ring kernel."""
    C = _native.require("gemm_xl_conv")
    torch.manual_seed(11)
    M, N, K = 5000, 512, 576
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    kw = {}
    if mode == "bnbwd":
        x = torch.randn(M, N, device=DEV).bfloat16()
        kw = dict(bn_x=x, mean=torch.zeros(N, device=DEV), invstd=torch.ones(N, device=DEV))
    C.set_gemm_xl_bn(256, 1)
    try:
        ref, rs = C.gemm_xl_conv(a, b, mode, **kw)
        C.set_gemm_xl_bn(256, pipe)
        got, gs = C.gemm_xl_conv(a, b, mode, **kw)
    finally:
        C.set_gemm_xl_bn(0)
    torch.testing.assert_close(got.float(), ref.float(), atol=0.02, rtol=1e-2)
    torch.testing.assert_close(gs, rs, atol=1e-2 * M ** 0.5, rtol=1e-3)
