"""MobileNetV2 inverted-residual block: the shortcut's gradient of x absorbed
into the expand conv's data-gradient GEMM (GradSlot) == the autograd engine's
separate add."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cin,cout", [(32, 32), (16, 24)])
def test_shortcut_grad_fused_into_expand_dgrad(cin, cout):
    from distributed_model_parallel_amd.models import mobilenetv2 as mv
    from distributed_model_parallel_amd.ops import conv1x1
    torch.manual_seed(0)
    blk = mv.InvertedResidual(cin, cout, 6, 1).cuda().bfloat16().to(memory_format=torch.channels_last).train()
    ref = copy.deepcopy(blk)
    x = torch.randn(16, cin, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    xa, xb = x.detach().requires_grad_(), x.detach().requires_grad_()
    n0 = conv1x1._STATS["fused_dgrad"]
    ya = blk(xa)
    old = mv._FUSE_SHORTCUT_GRAD
    mv._FUSE_SHORTCUT_GRAD = False
    try:
        yb = ref(xb)
    finally:
        mv._FUSE_SHORTCUT_GRAD = old
    torch.testing.assert_close(ya.float(), yb.float(), atol=0, rtol=0)
    g = torch.randn_like(ya)
    ya.backward(g)
    n1 = conv1x1._STATS["fused_dgrad"]
    yb.backward(g)
    assert n1 > n0
    err = (xa.grad.float() - xb.grad.float()).norm() / xb.grad.float().norm()
    assert err < 1e-2, err
    for (na, pa), (_, pb) in zip(blk.named_parameters(), ref.named_parameters()):
        e = (pa.grad.float() - pb.grad.float()).norm() / pb.grad.float().norm().clamp_min(1e-12)
        assert e < 2e-2, (na, e.item())
