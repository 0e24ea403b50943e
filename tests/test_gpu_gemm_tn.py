"""Split-M MFMA weight-gradient GEMM (transposing LDS reads) vs fp32 torch,
and the full native 1x1-conv autograd path vs F.conv2d."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops.conv1x1 import _STATS, Conv1x1

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(802816, 256, 64), (5000, 64, 256), (777, 128, 128), (64, 64, 64),
                                   (12544, 2048, 512), (100, 24, 144), (33, 8, 16)])
@pytest.mark.parametrize("out", [torch.float32, torch.bfloat16])
def test_gemm_tn(M, N, K, out):
    C = _native.require("gemm_tn")
    torch.manual_seed(0)
    a = torch.randn(M, N, device=DEV).bfloat16()
    b = torch.randn(M, K, device=DEV).bfloat16()
    got = C.gemm_tn(a, b, out)
    ref = a.float().t() @ b.float()
    tol = 1e-3 * M ** 0.5 + (0.02 * ref.abs().max().item() if out == torch.bfloat16 else 0)
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=1e-2)


def test_gemm_tn_asymmetric_pattern():
    """Exact small-integer data: any transpose/mapping slip changes the result."""
    C = _native.require("gemm_tn")
    M, N, K = 96, 64, 80
    a = (torch.arange(M * N, device=DEV).reshape(M, N) % 7 - 3).bfloat16()
    b = (torch.arange(M * K, device=DEV).reshape(M, K) % 5 - 2).bfloat16()
    torch.testing.assert_close(C.gemm_tn(a, b, torch.float32), a.float().t() @ b.float())


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_autograd_matches_conv2d(stride):
    torch.manual_seed(1)
    m = Conv1x1(64, 128, stride).cuda().bfloat16()
    x = torch.randn(4, 64, 14, 14, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    xi = x.detach().requires_grad_()
    n0 = _STATS["native"]
    y = m(xi)
    assert _STATS["native"] == n0 + 1
    yr = F.conv2d(xr, wr, None, stride)
    torch.testing.assert_close(y.float(), yr, atol=0.1, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=0.1, rtol=2e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=0.5, rtol=2e-2)


@pytest.mark.parametrize("hw", [(14, 14), (15, 9), (7, 8)])
def test_strided_row_maps(hw):
    """a_map (strided A read), c_map (strided scatter into zeros), b_map (strided wgrad
    operand) against explicit subsample / scatter in fp32."""
    C = _native.require("gemm_nt")
    torch.manual_seed(2)
    n, h, w, cin, cout, s = 3, hw[0], hw[1], 64, 96, 2
    ho, wo = (h - 1) // s + 1, (w - 1) // s + 1
    geom = [s, ho, wo, h, w]
    x = torch.randn(n, h, w, cin, device=DEV).bfloat16()
    wt = torch.randn(cout, cin, device=DEV).bfloat16()
    xs = x[:, ::s, ::s].reshape(-1, cin)
    y, _ = C.gemm_nt(x.reshape(-1, cin), wt, a_map=geom)
    torch.testing.assert_close(y.float(), xs.float() @ wt.float().t(), atol=0.1, rtol=2e-2)
    ym, mom = C.gemm_nt(x.reshape(-1, cin), wt, mode="moments", a_map=geom)
    yf = ym.float()
    torch.testing.assert_close(mom[:cout].float(), yf.sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    assert mom[-1].item() == n * ho * wo
    dy = torch.randn(n * ho * wo, cout, device=DEV).bfloat16()
    dx, _ = C.gemm_nt(dy, wt.t().contiguous(), c_map=geom)
    ref = torch.zeros(n, h, w, cin, device=DEV)
    ref[:, ::s, ::s] = (dy.float() @ wt.float()).view(n, ho, wo, cin)
    torch.testing.assert_close(dx.float().view(n, h, w, cin), ref, atol=0.1, rtol=2e-2)
    dw = C.gemm_tn(dy, x.reshape(-1, cin), torch.float32, b_map=geom)
    torch.testing.assert_close(dw, dy.float().t() @ xs.float(), atol=1e-3 * dy.shape[0] ** 0.5, rtol=1e-2)


def test_conv1x1_stride2_odd_spatial():
    torch.manual_seed(3)
    m = Conv1x1(32, 64, 2).cuda().bfloat16()
    x = torch.randn(2, 32, 9, 11, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    y = m(xi)
    yr = F.conv2d(xr, wr, None, 2)
    torch.testing.assert_close(y.float(), yr, atol=0.1, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=0.1, rtol=2e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=0.5, rtol=2e-2)


def test_gemm_tn_b_prologue():
    """B' = relu(B*s + t) per column, applied while staging (bn_relu_conv1x1 weight grad)."""
    C = _native.require("gemm_tn")
    torch.manual_seed(5)
    M, N, K = 3000, 64, 192
    a = torch.randn(M, N, device=DEV).bfloat16()
    b = torch.randn(M, K, device=DEV).bfloat16()
    s = torch.rand(K, device=DEV) + 0.5
    t = torch.randn(K, device=DEV) * 0.2
    got = C.gemm_tn(a, b, torch.float32, pro_scale=s, pro_shift=t)
    bp = torch.relu(b.float() * s + t).bfloat16().float()
    torch.testing.assert_close(got, a.float().t() @ bp, atol=1e-3 * M ** 0.5, rtol=1e-2)


@pytest.mark.parametrize("M,N,K", [(5000, 200, 768), (131, 128, 256), (40000, 512, 2304)])
def test_gemm_tn_wide_tile(M, N, K):
    """128 x 256 tiles (deep weight gradients) vs the fp32 reference, ragged N edge."""
    C = _native.require("gemm_tn")
    torch.manual_seed(6)
    a = torch.randn(M, N, device=DEV).bfloat16()
    b = torch.randn(M, K, device=DEV).bfloat16()
    ref = a.float().t() @ b.float()
    C.set_tn_wide(True)
    got = C.gemm_tn(a, b, torch.float32)
    C.set_tn_wide(False)
    try:
        narrow = C.gemm_tn(a, b, torch.float32)
    finally:
        C.set_tn_wide(True)
    tol = 1e-3 * M ** 0.5
    torch.testing.assert_close(got, ref, atol=tol, rtol=1e-2)
    torch.testing.assert_close(got, narrow, atol=tol, rtol=1e-2)


def test_conv_wgrad_wide_tile_3x3():
    """Implicit-GEMM 3x3 weight gradient with Cin % 256 == 0 (wide tile, one tap per K tile)."""
    C = _native.require("conv_wgrad")
    torch.manual_seed(7)
    n, cin, cout, h = 4, 256, 192, 9
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, h, h, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
    got = C.conv_wgrad(dy2, x, 3, 3, 1, 1, h, h, torch.float32).view(cout, 3, 3, cin).permute(0, 3, 1, 2)
    xr = x.float().requires_grad_()
    wr = torch.zeros(cout, cin, 3, 3, device=DEV, requires_grad=True)
    F.conv2d(xr, wr, None, 1, 1).backward(dy.float())
    torch.testing.assert_close(got, wr.grad, atol=1e-3 * (n * h * h) ** 0.5, rtol=1e-2)
