"""Halo-tiled 3x3 weight-gradient kernel (csrc/conv/wgrad3x3.hip) vs the fp32
PyTorch weight gradient of the same conv, on every ResNet-50 stride-1 3x3
shape family (64 ch @ 56, 128 @ 28, 256 @ 14, 512 @ 7), including partial
multi-image groups and row tiles."""
import pytest
import torch

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu


def _ref(dy, x, stride=1):
    return torch.nn.grad.conv2d_weight(x.float(), (dy.shape[1], x.shape[1], 3, 3), dy.float(), stride, 1)


@pytest.mark.parametrize("waves", [8, 4])
@pytest.mark.parametrize("n,c,h", [(2, 64, 56), (3, 64, 56), (2, 128, 28), (3, 256, 14), (5, 512, 7),
                                   (8, 512, 7), (1, 128, 28)])
def test_wgrad3x3_matches_fp32(n, c, h, waves):
    C = _native.require("wgrad3x3")
    C.set_wgrad3x3_waves(waves)
    assert C.wgrad3x3_supported(c, h, h)
    g = torch.Generator(device="cuda").manual_seed(n * 1000 + c)
    x = torch.randn(n, c, h, h, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(n, c, h, h, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = C.wgrad3x3(dy, x)
    assert out.shape == (c, c, 3, 3) and out.is_contiguous(memory_format=torch.channels_last)
    ref = _ref(dy, x)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    # bf16 output rounding (2^-8 relative) dominates; accumulation is fp32
    assert err <= 1e-2 * scale, (err, scale)
    # asymmetric data: the transpose of dW (co <-> ci swapped) must NOT match
    assert (out.float() - ref.transpose(0, 1)).abs().max().item() > 0.1 * scale
    C.set_wgrad3x3_waves(8)


def test_wgrad3x3_deterministic_and_zero_padding():
    C = _native.require("wgrad3x3")
    x = torch.ones(2, 64, 56, 56, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.ones_like(x)
    out = C.wgrad3x3(dy, x).float()
    # every (co, ci) sees, per tap, the number of output pixels whose tapped input is inside
    taps = torch.tensor([[55 * 55, 55 * 56, 55 * 55], [56 * 55, 56 * 56, 56 * 55], [55 * 55, 55 * 56, 55 * 55]],
                        device="cuda", dtype=torch.float32) * 2
    torch.testing.assert_close(out, taps.expand(64, 64, 3, 3), rtol=4e-3, atol=0)
    a = C.wgrad3x3(dy, x)
    b = C.wgrad3x3(dy, x)
    assert torch.equal(a, b)


def test_conv_module_backward_uses_halo_wgrad():
    """ResNet's 3x3/s1 ConvIG2d routes its weight gradient to the halo kernel
    (no MIOpen wrw) and matches the fp32 weight gradient."""
    import torch.nn.functional as F
    from distributed_model_parallel_amd.ops.conv_igemm import _STATS, ConvIG2d
    torch.manual_seed(3)
    m = ConvIG2d(128, 128, 3, 1, 1).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(4, 128, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = _STATS["halo_wgrad"]
    y = m(x)
    g = torch.randn_like(y)
    y.backward(g)
    assert _STATS["halo_wgrad"] == n0 + 1
    wr = m.weight.detach().float().requires_grad_()
    F.conv2d(x.float(), wr, None, 1, 1).backward(g.float())
    err = (m.weight.grad.float() - wr.grad).norm() / wr.grad.norm()
    assert err < 1e-2, err


@pytest.mark.parametrize("n,c,ho", [(2, 128, 28), (3, 256, 14)])
def test_wgrad3x3_stride2_matches_fp32(n, c, ho):
    """Stride-2 first blocks (column-deinterleaved halo): l2 / l3 shapes."""
    C = _native.require("wgrad3x3")
    assert C.wgrad3x3_supported(c, ho, ho, 2)
    g = torch.Generator(device="cuda").manual_seed(n * 7 + c)
    x = torch.randn(n, c, 2 * ho, 2 * ho, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(n, c, ho, ho, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    out = C.wgrad3x3(dy, x, 2)
    ref = _ref(dy, x, 2)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1e-2 * scale, (err, scale)
    assert (out.float() - ref.transpose(0, 1)).abs().max().item() > 0.1 * scale


@pytest.mark.parametrize("cin,h,stride", [(128, 28, 1), (128, 56, 2), (256, 28, 2), (64, 56, 1)])
def test_conv_module_input_and_weight_grads_together(cin, h, stride):
    """MIOpen data gradient + halo weight gradient in ONE backward (activations
    require grad, as inside the model): both gradients must arrive."""
    import torch.nn.functional as F
    from distributed_model_parallel_amd.ops.conv_igemm import _STATS, ConvIG2d
    torch.manual_seed(5)
    m = ConvIG2d(cin, cin, 3, stride, 1).cuda().bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, h, h, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    n0 = _STATS["halo_wgrad"]
    y = m(xi)
    g = torch.randn_like(y)
    y.backward(g)
    assert _STATS["halo_wgrad"] == n0 + 1
    assert m.weight.grad is not None and xi.grad is not None
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    F.conv2d(xr, wr, None, stride, 1).backward(g.float())
    for got, ref in ((m.weight.grad, wr.grad), (xi.grad, xr.grad)):
        err = (got.float() - ref).norm() / ref.norm()
        assert err < 1e-2, err
