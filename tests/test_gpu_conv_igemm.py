"""Implicit-GEMM MFMA convolution (forward + BN moments, transposed data
gradient, tap-gather weight gradient) vs an fp32 F.conv2d reference."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops.conv_igemm import _STATS, ConvIG2d, _wmat
from distributed_model_parallel_amd.ops.conv_igemm import conv2d_igemm as conv_igemm_fn

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHAPES = [  # n, cin, cout, h, w, k, stride, pad
    (2, 64, 64, 14, 14, 3, 1, 1),
    (2, 64, 128, 15, 13, 3, 2, 1),
    (3, 128, 64, 7, 9, 3, 1, 1),
    (2, 192, 64, 8, 8, 3, 2, 1),
    (1, 64, 64, 5, 6, 1, 2, 0),
    (2, 128, 128, 6, 6, 3, 1, 0),
]


@pytest.fixture(autouse=True)
def _native_forward(monkeypatch):
    """These tests exercise our kernels: keep layer-1/2-sized forwards off MIOpen."""
    from distributed_model_parallel_amd.ops import conv_igemm
    monkeypatch.setattr(conv_igemm, "_MIOPEN_FWD", False)


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_forward_and_moments(shape):
    C = _native.require("conv_nt")
    n, cin, cout, h, w, k, s, p = shape
    torch.manual_seed(0)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).bfloat16())
    wt = _cl(torch.randn(cout, cin, k, k, device=DEV).bfloat16() * 0.1)
    ref = F.conv2d(x.float(), wt.float(), None, s, p)
    ho, wo = ref.shape[2:]
    y, _ = C.conv_nt(x, _wmat(wt), k, k, s, p, ho, wo)
    got = y.float().view(n, ho, wo, cout).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=0.05, rtol=2e-2)
    ym, mom = C.conv_nt(x, _wmat(wt), k, k, s, p, ho, wo, mode="moments")
    yf = ym.float()
    torch.testing.assert_close(mom[:cout].float(), yf.sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    torch.testing.assert_close(mom[cout:2 * cout].float(), (yf * yf).sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    assert mom[-1].item() == n * ho * wo


@pytest.fixture(params=[True, False], ids=["native_bwd", "miopen_bwd"])
def bwd_mode(request):
    from distributed_model_parallel_amd.ops import conv_igemm
    old = conv_igemm.NATIVE_BWD
    conv_igemm.NATIVE_BWD = request.param
    yield request.param
    conv_igemm.NATIVE_BWD = old


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_autograd(shape, bwd_mode):
    n, cin, cout, h, w, k, s, p = shape
    torch.manual_seed(1)
    m = ConvIG2d(cin, cout, k, s, p).to(DEV).bfloat16().to(memory_format=torch.channels_last)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).bfloat16())
    xi = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    n0 = _STATS["native"]
    y = m(xi)
    assert _STATS["native"] == n0 + 1
    yr = F.conv2d(xr, wr, None, s, p)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=0.1, rtol=2e-2)
    rows = n * yr.shape[2] * yr.shape[3]
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=0.05 * rows ** 0.5, rtol=2e-2)


def test_conv_wgrad_exact_pattern():
    """Small-integer data: any tap / transpose mapping slip changes the result exactly."""
    C = _native.require("conv_wgrad")
    n, cin, cout, h, w = 2, 64, 64, 6, 5
    x = _cl((torch.arange(n * cin * h * w, device=DEV).reshape(n, cin, h, w) % 5 - 2).bfloat16())
    dy = (torch.arange(n * 3 * 3 * cout, device=DEV).reshape(n * 9, cout) % 3 - 1).bfloat16()
    got = C.conv_wgrad(dy, x, 3, 3, 2, 1, 3, 3, torch.float32).view(cout, 3, 3, cin).permute(0, 3, 1, 2)
    xr = x.float().requires_grad_(False)
    wr = torch.zeros(cout, cin, 3, 3, device=DEV, requires_grad=True)
    out = F.conv2d(xr, wr, None, 2, 1)
    out.backward(dy.float().view(n, 3, 3, cout).permute(0, 3, 1, 2))
    torch.testing.assert_close(got, wr.grad)


@pytest.mark.parametrize("shape", [(16, 64, 64, 56, 56, 3, 1, 1), (16, 128, 128, 56, 56, 3, 2, 1),
                                   (32, 256, 256, 14, 14, 3, 1, 1), (32, 512, 512, 14, 14, 3, 2, 1)])
def test_conv_large_resnet_shapes(shape, bwd_mode):
    """ResNet-50 layer shapes at a realistic M: many M tiles, many wgrad splits."""
    n, cin, cout, h, w, k, s, p = shape
    torch.manual_seed(4)
    x = _cl(torch.randn(n, cin, h, w, device=DEV).bfloat16())
    wt = _cl((torch.randn(cout, cin, k, k, device=DEV) * (2.0 / (cin * k * k)) ** 0.5).bfloat16())
    xi = x.detach().requires_grad_()
    wi = wt.detach().requires_grad_()
    y, _ = conv_igemm_fn(xi, wi, s, p)
    xr = x.detach().float().requires_grad_()
    wr = wt.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, s, p)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for got, ref, name in ((y.float(), yr, "y"), (xi.grad.float(), xr.grad, "dx"), (wi.grad.float(), wr.grad, "dw")):
        err = (got - ref).norm() / ref.norm()
        assert err < 1e-2, f"{name}: relative error {err:.4g}"


@pytest.mark.parametrize("n,c,h", [(3, 256, 28), (2, 512, 14), (5, 256, 6)])
def test_xl_stride2_phase_dgrad(n, c, h):
    """Stride-2 3x3 data gradient of layers 3-4 as four stride-phase ping-pong
    GEMMs (gemm_xl.hip conv_xl_dgrad_s2) vs fp32 autograd, through the module
    path and through the kernel directly."""
    from distributed_model_parallel_amd.ops import conv_igemm
    C = _native.require("conv_xl_dgrad_s2")
    torch.manual_seed(7)
    x = _cl(torch.randn(n, c, h, h, device=DEV).bfloat16())
    wt = _cl((torch.randn(c, c, 3, 3, device=DEV) * (2.0 / (c * 9)) ** 0.5).bfloat16())
    xr = x.detach().float().requires_grad_()
    yr = F.conv2d(xr, wt.float(), None, 2, 1)
    g = torch.randn_like(yr)
    yr.backward(g)
    dy = _cl(g.bfloat16())
    dx = C.conv_xl_dgrad_s2(dy, conv_igemm._phase_weights(wt), h, h).view(n, h, h, c).permute(0, 3, 1, 2)
    err = ((dx.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert err < 1e-2, err
    xi = x.detach().requires_grad_()
    wi = wt.detach().requires_grad_()
    n0 = _STATS["xl_dgrad_s2"]
    y, _ = conv_igemm_fn(xi, wi, 2, 1)
    y.backward(dy)
    assert _STATS["xl_dgrad_s2"] == n0 + 1
    err2 = ((xi.grad.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert err2 < 1e-2, err2
