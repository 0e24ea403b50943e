"""Native Linear side passes (csrc/linear/bias_act.hip) against fp32 PyTorch:
bias gradient column sums and the fused GELU backward + bias gradient, at
ViT-B/16 widths (768, 2304, 3072) and odd row counts; plus the ViT MLP
through ops/linear.py."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops import linear as L

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N", [(25216, 768), (1000, 2304), (37, 3072), (1, 256), (4099, 512)])
def test_bias_grad(M, N):
    C = _native.require("bias_grad test")
    torch.manual_seed(0)
    dy = torch.randn(M, N, device=DEV).bfloat16()
    ref = dy.float().sum(0)
    for dt in (torch.bfloat16, torch.float32):
        got = C.bias_grad(dy, dt)
        assert got.dtype == dt
        torch.testing.assert_close(got.float(), ref, atol=2e-2 * (M ** 0.5) / 10 + 1e-2, rtol=1e-2)


@pytest.mark.parametrize("M,N", [(25216, 3072), (333, 768), (8, 512)])
def test_gelu_bwd_bias_grad(M, N):
    C = _native.require("gelu bwd test")
    torch.manual_seed(1)
    h = (torch.randn(M, N, device=DEV) * 2).bfloat16()
    dy = torch.randn(M, N, device=DEV).bfloat16()
    hr = h.float().requires_grad_()
    F.gelu(hr).backward(dy.float())
    dh, db = C.gelu_bwd_bias_grad(dy, h, torch.bfloat16)
    torch.testing.assert_close(dh.float(), hr.grad, atol=2e-2, rtol=2e-2)
    # the bias gradient is the exact column sum of the stored (bf16) dh
    torch.testing.assert_close(db.float(), dh.float().sum(0), atol=0.5, rtol=1e-2)
    torch.testing.assert_close(db.float(), hr.grad.sum(0), atol=1.0 + 0.02 * M ** 0.5, rtol=2e-2)


def test_linear_modules_match_torch():
    torch.manual_seed(2)
    x = torch.randn(4, 197, 768, device=DEV).bfloat16()
    lin = L.Linear(768, 2304).to(DEV).bfloat16()
    w, b = lin.weight.detach().float().requires_grad_(), lin.bias.detach().float().requires_grad_()
    xr = x.float().requires_grad_()
    xn = x.clone().requires_grad_()
    n0 = L._STATS["native"]
    y = lin(xn)
    g = L.linear_gelu(y, torch.randn(512, 2304, device=DEV).bfloat16(), torch.zeros(512, device=DEV).bfloat16())
    assert L._STATS["native"] == n0 + 2
    yr = F.linear(xr, w, b)
    torch.testing.assert_close(y.float(), yr, atol=6e-2, rtol=2e-2)
    gy = torch.randn_like(yr)
    y.backward(gy.bfloat16(), retain_graph=True)
    yr.backward(gy)
    torch.testing.assert_close(lin.bias.grad.float(), b.grad, atol=0.3, rtol=2e-2)
    rel = (lin.weight.grad.float() - w.grad).norm() / w.grad.norm()
    assert rel < 2e-2
    rel = (xn.grad.float() - xr.grad).norm() / xr.grad.norm()
    assert rel < 2e-2
    assert torch.isfinite(g).all()


def test_vit_mlp_native_vs_reference():
    from distributed_model_parallel_amd.models.vit import MLP
    torch.manual_seed(3)
    mlp = MLP(768, 3072).to(DEV).bfloat16()
    x = torch.randn(2, 197, 768, device=DEV).bfloat16().requires_grad_()
    y = mlp(x)
    xr = x.detach().float().requires_grad_()
    w1, b1 = mlp.fc1.weight.float().detach().requires_grad_(), mlp.fc1.bias.float().detach().requires_grad_()
    w2, b2 = mlp.fc2.weight.float().detach().requires_grad_(), mlp.fc2.bias.float().detach().requires_grad_()
    yr = F.linear(F.gelu(F.linear(xr, w1, b1)), w2, b2)
    torch.testing.assert_close(y.float(), yr, atol=5e-2, rtol=5e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    for got, ref in ((mlp.fc1.bias.grad, b1.grad), (mlp.fc2.bias.grad, b2.grad),
                     (mlp.fc1.weight.grad, w1.grad), (x.grad, xr.grad)):
        rel = (got.float() - ref).norm() / ref.norm()
        assert rel < 3e-2, rel
