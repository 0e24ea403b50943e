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


def test_stem_bn_pool_fusion_matches_unfused():
    """conv_bn_maxpool: BN+ReLU inside the pool (forward) and the BN backward's
    reductions inside the pool's backward == the three modules run separately."""
    import copy

    from distributed_model_parallel_amd.ops import fused
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
    from distributed_model_parallel_amd.ops.pool import MaxPool2d
    torch.manual_seed(0)
    conv = StemConv2d(3, 64).cuda().bfloat16().to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(64, act="relu").cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0.0, 0.2)
    pool = MaxPool2d(3, 2, 1)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(4, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = fused._STATS_FUSED["bn_relu_maxpool"]
    y = fused.conv_bn_maxpool(conv, bn, pool, x)
    assert fused._STATS_FUSED["bn_relu_maxpool"] == n0 + 1, "fused stem did not run"
    old = fused._FUSE_STEM_POOL
    fused._FUSE_STEM_POOL = False
    try:
        yr = fused.conv_bn_maxpool(conv2, bn2, pool, x)
    finally:
        fused._FUSE_STEM_POOL = old
    torch.testing.assert_close(y.float(), yr.float())
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for a, b, name in ((conv.weight.grad, conv2.weight.grad, "conv w"), (bn.weight.grad, bn2.weight.grad, "bn w"),
                       (bn.bias.grad, bn2.bias.grad, "bn b")):
        err = (a.float() - b.float()).norm() / b.float().norm()
        assert err < 2e-2, (name, err.item())
    torch.testing.assert_close(bn.running_mean, bn2.running_mean)
    torch.testing.assert_close(bn.running_var, bn2.running_var)
    assert int(bn.num_batches_tracked) == int(bn2.num_batches_tracked) == 1


@pytest.mark.parametrize("n,h,w,cout", [(8, 32, 32, 32), (3, 17, 13, 64)])
def test_rowtap_stem_matches_conv2d(n, h, w, cout):
    """MobileNetV2's 3x3/s1 stem on 3 channels as 64-channel row taps."""
    from distributed_model_parallel_amd.ops.stem import RowTapConv2d
    torch.manual_seed(1)
    m = RowTapConv2d(3, cout, 3).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(n, 3, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = _STATS["native"]
    y, mom = m.forward_with_moments(x)
    assert _STATS["native"] == n0 + 1
    wr = m.weight.detach().float().requires_grad_()
    yr = F.conv2d(x.float(), wr, None, 1, 1)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout).double()
    torch.testing.assert_close(mom[:cout], yf.sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    err = (m.weight.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert err < 1e-2, err


@pytest.mark.parametrize("n", [1, 7, 40])
def test_stem_halo_kernels_224(n):
    """224-px stem on the halo-tiled kernels (csrc/conv/stem_halo.hip): forward +
    moments and weight gradient vs fp32, several persistent tile ranges."""
    torch.manual_seed(n)
    m = StemConv2d(3, 64).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(n, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    h0 = _STATS["halo"]
    y, mom = m.forward_with_moments(x)
    assert _STATS["halo"] == h0 + 1, "halo stem did not run"
    wr = m.weight.detach().float().requires_grad_()
    yr = F.conv2d(x.float(), wr, None, 2, 3)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64).double()
    torch.testing.assert_close(mom[:64], yf.sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    torch.testing.assert_close(mom[64:128], (yf * yf).sum(0), atol=1e-2 * yf.shape[0] ** 0.5, rtol=1e-3)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    err = (m.weight.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert err < 1e-2, err
    # no-moments forward path too
    y2 = m(x)
    assert torch.equal(y2, y)


@pytest.mark.parametrize("shift", [0.0, 2.0])
def test_stem_bn_backward_folded_into_wgrad(shift):
    """224 px: the stem's BN backward apply folded into its weight gradient
    (ops/fused.py _StemBNReLUMaxPoolFn: dW = a dz^T P + b y^T P + c colsum P,
    no dx pass) == the pool-fused path that materialises dx.  ``shift`` moves
    the conv outputs' mean away from 0 (the b and c terms then cancel more)."""
    import copy

    from distributed_model_parallel_amd.ops import fused
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
    from distributed_model_parallel_amd.ops.pool import MaxPool2d
    torch.manual_seed(0)
    conv = StemConv2d(3, 64).cuda().bfloat16().to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(64, act="relu").cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.normal_(0.0, 0.2)
    pool = MaxPool2d(3, 2, 1)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = (torch.randn(8, 3, 224, 224, device="cuda") + shift).bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = fused._STATS_FUSED["stem_bn_relu_maxpool"]
    y = fused.conv_bn_maxpool(conv, bn, pool, x)
    assert fused._STATS_FUSED["stem_bn_relu_maxpool"] == n0 + 1, "folded stem did not run"
    old = fused._FUSE_STEM_WGRAD
    fused._FUSE_STEM_WGRAD = False
    try:
        yr = fused.conv_bn_maxpool(conv2, bn2, pool, x)
    finally:
        fused._FUSE_STEM_WGRAD = old
    assert fused._STATS_FUSED["stem_bn_relu_maxpool"] == n0 + 1
    torch.testing.assert_close(y.float(), yr.float())
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    for a, b, name in ((conv.weight.grad, conv2.weight.grad, "conv w"), (bn.weight.grad, bn2.weight.grad, "bn w"),
                       (bn.bias.grad, bn2.bias.grad, "bn b")):
        err = (a.float() - b.float()).norm() / b.float().norm()
        # the reference rounds dx to bf16 before its weight gradient; the fold does not
        assert err < 2e-2, (name, err.item())
    torch.testing.assert_close(bn.running_var, bn2.running_var)


@pytest.mark.parametrize("n,c,h,w", [(3, 64, 16, 16), (2, 32, 14, 10), (2, 64, 9, 11), (1, 128, 8, 8)])
def test_bn_pool_backward_kernel_vs_fp32(n, c, h, w):
    """maxpool2d_bn_backward (quad kernel for even H/W, one-pixel kernel for odd)
    against an fp32 scatter of dy through the forward's argmax taps."""
    from distributed_model_parallel_amd import _native
    C = _native.require("bn pool backward")
    torch.manual_seed(0)
    x = torch.randn(n, c, h, w, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    sc = (torch.rand(c, device="cuda") + 0.5).contiguous()
    sh = (torch.randn(c, device="cuda") * 0.3).contiguous()
    mean = (torch.randn(c, device="cuda") * 0.1).contiguous()
    y, idx = C.maxpool2d_bn_forward(x, sc, sh, 3, 2, 1)
    ho, wo = y.shape[2], y.shape[3]
    dy = torch.randn(n, c, ho, wo, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    dz, sums = C.maxpool2d_bn_backward(dy, idx, x, sc, sh, mean, 3, 2, 1)
    # reference: output (oh, ow) sends dy to input (2oh-1+a, 2ow-1+b), tap = 3a+b
    tap = idx.view(n, ho, wo, c).long()
    oh = torch.arange(ho, device="cuda").view(1, ho, 1, 1)
    ow = torch.arange(wo, device="cuda").view(1, 1, wo, 1)
    ih = 2 * oh - 1 + tap // 3
    iw = 2 * ow - 1 + tap % 3
    assert bool(((ih >= 0) & (ih < h) & (iw >= 0) & (iw < w)).all())
    nn_ = torch.arange(n, device="cuda").view(n, 1, 1, 1).expand_as(tap)
    cc = torch.arange(c, device="cuda").view(1, 1, 1, c).expand_as(tap)
    flat = ((nn_ * h + ih) * w + iw) * c + cc
    g = torch.zeros(n * h * w * c, device="cuda")
    g.index_add_(0, flat.reshape(-1), dy.permute(0, 2, 3, 1).reshape(-1).float())
    g = g.view(n, h, w, c).bfloat16().float()
    xf = x.permute(0, 2, 3, 1).float()
    dref = torch.where(xf * sc + sh > 0, g, torch.zeros_like(g))
    torch.testing.assert_close(dz.permute(0, 2, 3, 1).float(), dref, atol=0, rtol=0)
    d64 = dref.double().reshape(-1, c)
    torch.testing.assert_close(sums[:c], d64.sum(0), atol=1e-3, rtol=1e-4)
    torch.testing.assert_close(sums[c:2 * c], (d64 * (xf.double().reshape(-1, c) - mean.double())).sum(0),
                               atol=1e-3, rtol=1e-4)
    assert sums[2 * c].item() == n * h * w
