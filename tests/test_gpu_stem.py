"""Space-to-depth MFMA stem conv (ops/stem.py, csrc/conv/stem.hip) vs an fp32
F.conv2d reference: output, fused BN moments, weight gradient."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.stem import _STATS, StemConv2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,h,w", [(4, 224, 224), (3, 64, 48), (2, 31, 37)])
def test_stem_forward_moments_wgrad(n, h, w):
    torch.manual_seed(0)
    m = StemConv2d(3, 64).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(n, 3, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = _STATS["native"]
    y, mom = m.forward_with_moments(x)
    assert _STATS["native"] == n0 + 1, "native stem did not run"
    wr = m.weight.detach().float().requires_grad_()
    yr = F.conv2d(x.float(), wr, None, 2, 3)
    assert y.shape == yr.shape
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64).double()
    torch.testing.assert_close(mom[:64], yf.sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    torch.testing.assert_close(mom[64:128], (yf * yf).sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    assert mom[128].item() == yf.shape[0]
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    err = (m.weight.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert err < 1e-2, err


def test_stem_falls_back_when_input_needs_grad():
    m = StemConv2d(3, 64).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(2, 3, 32, 32, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    n0 = _STATS["torch"]
    m(x).sum().backward()
    assert _STATS["torch"] == n0 + 1 and x.grad is not None
