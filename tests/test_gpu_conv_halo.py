"""Halo-tiled 3x3 convs (64->64: csrc/conv/conv3x3_halo.hip; 128->128:
conv3x3_c128.hip) against an fp32
PyTorch reference: forward, fused BN moments, and the data gradient through
ops.conv_igemm (same kernel over flipped weights).  H covers whole tiles (56),
a partial last tile (10: 4 + 4 + 2 rows) and a single partial tile (3)."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops import conv_igemm

pytestmark = pytest.mark.gpu


def _inputs(n, h, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, 64, h, 56, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, generator=g) * (1.0 / 24)).cuda().bfloat16() \
        .contiguous(memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("n,h", [(2, 56), (3, 10), (5, 3), (300, 8)])
def test_halo_forward_and_moments(n, h):
    C = _native.require("test")
    x, w = _inputs(n, h)
    ref = F.conv2d(x.float(), w.float(), None, 1, 1)
    y2, mom = C.conv3x3_c64(x, conv_igemm._wmat(w).contiguous(), True)
    y = y2.view(n, h, 56, 64).permute(0, 3, 1, 2).float()
    err = (y - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item() + 1e-2, err
    # moments of the bf16 output the kernel stored
    yb = y2.double()
    assert mom.shape == (129,)
    torch.testing.assert_close(mom[:64], yb.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(mom[64:128], (yb * yb).sum(0), rtol=1e-4, atol=1e-2)
    assert mom[128].item() == n * h * 56
    y3, m3 = C.conv3x3_c64(x, conv_igemm._wmat(w).contiguous(), False)
    assert torch.equal(y3, y2) and m3.numel() == 0


def test_halo_routing_fwd_bwd():
    n, h = 4, 56
    x, w = _inputs(n, h, seed=1)
    xr = x.float().clone().requires_grad_(True)
    wr = w.float().clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, 1, 1)
    g = torch.randn_like(ref)
    ref.backward(g)
    x.requires_grad_(True)
    before = dict(conv_igemm._STATS)
    y, mom = conv_igemm.conv2d_igemm(x, w.requires_grad_(True), 1, 1, moments=True)
    y.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    assert conv_igemm._STATS["halo_fwd"] == before["halo_fwd"] + 1
    assert conv_igemm._STATS["halo_dgrad"] == before["halo_dgrad"] + 1
    assert (y.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2
    dx_err = (x.grad.float() - xr.grad).abs().max().item()
    assert dx_err < 2e-2 * xr.grad.abs().max().item() + 1e-2, dx_err
    cos = F.cosine_similarity(w.grad.float().flatten(), wr.grad.flatten(), dim=0).item()
    assert cos > 0.999, cos


# ---- 128 -> 128 on 28-wide maps (csrc/conv/conv3x3_c128.hip) ----

def _inputs128(n, h, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(n, 128, h, 28, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 3, 3, generator=g) * (1.0 / 34)).cuda().bfloat16() \
        .contiguous(memory_format=torch.channels_last)
    return x, w


@pytest.mark.parametrize("n,h", [(2, 28), (3, 8), (1, 4), (301, 4)])
def test_c128_forward_and_moments(n, h):
    C = _native.require("test")
    x, w = _inputs128(n, h)
    ref = F.conv2d(x.float(), w.float(), None, 1, 1)
    y2, mom = C.conv3x3_c128(x, conv_igemm._wmat(w).contiguous(), True)
    y = y2.view(n, h, 28, 128).permute(0, 3, 1, 2).float()
    err = (y - ref).abs().max().item()
    assert err < 2e-2 * ref.abs().max().item() + 1e-2, err
    yb = y2.double()
    assert mom.shape == (257,)
    torch.testing.assert_close(mom[:128], yb.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(mom[128:256], (yb * yb).sum(0), rtol=1e-4, atol=1e-2)
    assert mom[256].item() == n * h * 28
    y3, m3 = C.conv3x3_c128(x, conv_igemm._wmat(w).contiguous(), False)
    assert torch.equal(y3, y2) and m3.numel() == 0


def test_c128_routing_fwd_bwd():
    n, h = 4, 28
    x, w = _inputs128(n, h, seed=1)
    xr = x.float().clone().requires_grad_(True)
    wr = w.float().clone().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, 1, 1)
    g = torch.randn_like(ref)
    ref.backward(g)
    x.requires_grad_(True)
    before = dict(conv_igemm._STATS)
    y, mom = conv_igemm.conv2d_igemm(x, w.requires_grad_(True), 1, 1, moments=True)
    y.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    assert conv_igemm._STATS["halo_fwd"] == before["halo_fwd"] + 1
    assert conv_igemm._STATS["halo_dgrad"] == before["halo_dgrad"] + 1
    assert conv_igemm._STATS["halo_wgrad"] == before["halo_wgrad"] + 1
    assert (y.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2
    dx_err = (x.grad.float() - xr.grad).abs().max().item()
    assert dx_err < 2e-2 * xr.grad.abs().max().item() + 1e-2, dx_err
    cos = F.cosine_similarity(w.grad.float().flatten(), wr.grad.flatten(), dim=0).item()
    assert cos > 0.999, cos
    # the plain (no-moments) forward module path takes the same kernel
    before = dict(conv_igemm._STATS)
    m = conv_igemm.ConvIG2d(128, 128, 3, 1, 1).cuda().bfloat16().to(memory_format=torch.channels_last)
    with torch.no_grad():
        m.weight.copy_(w)
        out = m(x.detach())
    assert conv_igemm._STATS["halo_fwd"] == before["halo_fwd"] + 1
    assert (out.float() - ref.detach()).abs().max().item() < 2e-2 * ref.abs().max().item() + 1e-2


@pytest.mark.parametrize("n,h", [(2, 28), (3, 4), (65, 8)])
def test_c128_stride2_phase_dgrad(n, h):
    """Layer-2 block-0 3x3/s2 data gradient (dy h x 28 -> dx 2h x 56) as four
    stride phases on the c128 halo kernel vs fp32 autograd, directly and
    through the module path."""
    C = _native.require("test")
    g = torch.Generator(device="cpu").manual_seed(3)
    x = torch.randn(n, 128, 2 * h, 56, generator=g).cuda().bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(128, 128, 3, 3, generator=g) * (1.0 / 34)).cuda().bfloat16() \
        .contiguous(memory_format=torch.channels_last)
    xr = x.float().clone().requires_grad_(True)
    yr = F.conv2d(xr, w.float(), None, 2, 1)
    gy = torch.randn(yr.shape, generator=g).cuda()
    yr.backward(gy)
    dy = gy.bfloat16().contiguous(memory_format=torch.channels_last)
    wt = w.permute(1, 2, 3, 0).reshape(128, -1).contiguous()
    dx = C.conv3x3_c128_dgrad_s2(dy, wt).view(n, 2 * h, 56, 128).permute(0, 3, 1, 2)
    err = ((dx.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert err < 1e-2, err
    assert (dx.float() - xr.grad).abs().max().item() < 2e-2 * xr.grad.abs().max().item() + 1e-2
    xi = x.detach().requires_grad_(True)
    before = dict(conv_igemm._STATS)
    y, _ = conv_igemm.conv2d_igemm(xi, w.detach().requires_grad_(True), 2, 1)
    y.backward(dy)
    assert conv_igemm._STATS["halo_dgrad_s2"] == before["halo_dgrad_s2"] + 1
    err2 = ((xi.grad.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert err2 < 1e-2, err2
