"""Implicit-GEMM convolution on the 256x256 ping-pong MFMA kernel (csrc/gemm/
gemm_xl.hip conv_xl: NHWC tap gather through LDS-DMA, padding taps from a
zero row) against fp32 F.conv2d: forward with and without the BN-moments
epilogue, stride 2, ragged Cout, and the stride-1 data gradient written as a
forward conv over flipped weights."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def wmat(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


@pytest.mark.parametrize("n,cin,cout,h,k,s", [(4, 64, 256, 9, 3, 1), (3, 128, 512, 15, 3, 2), (2, 256, 136, 7, 3, 1),
                                              (5, 64, 256, 8, 1, 1), (2, 192, 256, 11, 3, 2)])
def test_conv_xl_forward(n, cin, cout, h, k, s):
    C = _native.require("conv_xl")
    torch.manual_seed(0)
    p = k // 2
    ho = (h + 2 * p - k) // s + 1
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, k, k, device=DEV) * 0.05).bfloat16()
    ref = F.conv2d(x.float(), w.float(), None, s, p).permute(0, 2, 3, 1).reshape(-1, cout)
    y, _ = C.conv_xl(x, wmat(w), k, k, s, p, ho, ho, "store")
    torch.testing.assert_close(y.float(), ref, atol=0.05, rtol=2e-2)
    y2, sums = C.conv_xl(x, wmat(w), k, k, s, p, ho, ho, "moments")
    torch.testing.assert_close(y2, y)
    yf = y2.float()
    torch.testing.assert_close(sums[:cout].float(), yf.sum(0), atol=2e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    torch.testing.assert_close(sums[cout:2 * cout].float(), (yf * yf).sum(0), atol=2e-2 * yf.shape[0] ** 0.5,
                               rtol=1e-3)
    assert sums[-1].item() == n * ho * ho


def test_conv_xl_exact_pattern():
    """Small-integer data (exact in bf16 / fp32): any tap, channel or padding slip shows."""
    C = _native.require("conv_xl")
    n, cin, cout, h = 2, 64, 256, 6
    x = (torch.arange(n * cin * h * h, device=DEV).reshape(n, cin, h, h) % 5 - 2).bfloat16()
    x = x.contiguous(memory_format=CL)
    w = (torch.arange(cout * cin * 9, device=DEV).reshape(cout, cin, 3, 3) % 3 - 1).bfloat16()
    ref = F.conv2d(x.float(), w.float(), None, 1, 1).permute(0, 2, 3, 1).reshape(-1, cout)
    y, _ = C.conv_xl(x, wmat(w), 3, 3, 1, 1, h, h, "store")
    assert torch.equal(y.float(), ref)


@pytest.mark.parametrize("cin,cout,h", [(256, 256, 7), (128, 64, 10)])
def test_conv_xl_dgrad_as_flipped_conv(cin, cout, h):
    """dx of a 3x3/s1/p1 conv = conv(dy, flip(W)^T) with pad 1."""
    C = _native.require("conv_xl")
    torch.manual_seed(1)
    n = 3
    x = torch.randn(n, cin, h, h, device=DEV, requires_grad=True)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.05).bfloat16()
    dy = torch.randn(n, cout, h, h, device=DEV).bfloat16()
    F.conv2d(x, w.float(), None, 1, 1).backward(dy.float())
    wflip = w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, 9 * cout).contiguous()
    dx, _ = C.conv_xl(dy.contiguous(memory_format=CL), wflip, 3, 3, 1, 1, h, h, "store")
    torch.testing.assert_close(dx.float(), x.grad.permute(0, 2, 3, 1).reshape(-1, cin), atol=0.05, rtol=2e-2)
