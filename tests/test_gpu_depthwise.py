"""Native 3x3 depthwise conv (forward, data grad, weight grad, output moments)
against fp32 PyTorch conv2d(groups=C)."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops.depthwise import _STATS, DepthwiseConv2d

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("N,C,H,W,stride", [(4, 96, 32, 32, 1), (3, 144, 32, 32, 2), (2, 960, 4, 4, 1),
                                            (5, 8, 9, 7, 2), (2, 24, 7, 9, 1), (1, 384, 8, 8, 2),
                                            (2, 16, 1, 1, 1), (2, 16, 2, 3, 2), (3, 40, 6, 10, 2)])
def test_depthwise_fwd_bwd(dtype, N, C, H, W, stride):
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device=DEV).to(dtype).contiguous(memory_format=torch.channels_last)
    m = DepthwiseConv2d(C, stride).to(DEV)
    w32 = m.weight.detach().clone().float()
    m = m.to(dtype)
    xr = x.detach().float().requires_grad_()
    wr = w32.clone().requires_grad_()
    xi = x.detach().requires_grad_()
    before = _STATS["native"]
    y = m(xi)
    assert _STATS["native"] == before + 1
    yr = F.conv2d(xr, wr, None, stride, 1, 1, C)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    yr.backward(g)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=tol * 3, rtol=tol)
    wtol = 0.05 * (N * H * W / stride ** 2) ** 0.5 if dtype == torch.bfloat16 else 1e-2
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=wtol, rtol=tol * 3)


def test_depthwise_forward_moments():
    C = _native.require("dw")
    x = torch.randn(8, 64, 16, 16, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 1, 3, 3, device=DEV).bfloat16()
    y, mom = C.dwconv3x3_forward(x, w, 1, True)
    yf = y.float().double().permute(0, 2, 3, 1).reshape(-1, 64)
    torch.testing.assert_close(mom[:64], yf.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(mom[64:128], (yf * yf).sum(0), atol=1e-2, rtol=1e-4)
    assert mom[128].item() == 8 * 16 * 16


@pytest.mark.parametrize("wkind", ["fp32", "bf16_offset1", "fp32_offset2"])
def test_depthwise_weight_layouts(wkind):
    """The kernels read the [C,1,3,3] weight in place (bf16 or fp32, 16-B aligned);
    an fp32 weight with bf16 activations and a misaligned view (converted copy)
    give the same results as conv2d."""
    C = _native.require("dw")
    torch.manual_seed(0)
    n, c, h, w = 3, 48, 10, 12
    x = torch.randn(n, c, h, w, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    base = torch.randn(c * 9 + 8, device=DEV) * 0.3
    if wkind == "fp32":
        wt = base[: c * 9].view(c, 1, 3, 3)
    elif wkind == "bf16_offset1":
        wt = base.bfloat16()[1: 1 + c * 9].view(c, 1, 3, 3)
    else:
        wt = base[2: 2 + c * 9].view(c, 1, 3, 3)
    assert wkind == "fp32" or wt.data_ptr() % 16 != 0
    for stride in (1, 2):
        y, _ = C.dwconv3x3_forward(x, wt, stride, False)
        yr = F.conv2d(x.float(), wt.float(), None, stride, 1, 1, c)
        torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
        dy = torch.randn_like(yr).bfloat16().contiguous(memory_format=torch.channels_last)
        dx = C.dwconv3x3_dgrad(dy, wt, stride, h, w)
        xr = x.float().requires_grad_()
        F.conv2d(xr, wt.float(), None, stride, 1, 1, c).backward(dy.float())
        torch.testing.assert_close(dx.float(), xr.grad, atol=6e-2, rtol=3e-2)
        dw = C.dwconv3x3_wgrad(dy, x, stride, wt.dtype)
        assert dw.shape == (c, 1, 3, 3) and dw.dtype == wt.dtype and dw.is_contiguous()
        wr = wt.float().detach().requires_grad_()
        F.conv2d(x.float(), wr, None, stride, 1, 1, c).backward(dy.float())
        torch.testing.assert_close(dw.float(), wr.grad, atol=0.05 * (n * h * w) ** 0.5, rtol=5e-2)
