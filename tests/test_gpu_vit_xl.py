"""ViT encoder block on the fused-epilogue ping-pong GEMMs (ops/linear.py
mlp_residual / linear_residual) against the same math in fp32 PyTorch:
forward output and every gradient (input, residual, weights, biases)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_model_parallel_amd.ops import linear as L

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _xl_on(monkeypatch):
    monkeypatch.setattr(L, "_XL", True)


def _ref_mlp(x, res, w1, b1, w2, b2):
    return res + F.linear(F.gelu(F.linear(x, w1, b1)), w2, b2)


def _leaves(*ts):
    return [t.detach().clone().requires_grad_() for t in ts]


@pytest.mark.parametrize("T,D,H", [(8192, 256, 1024), (4100, 768, 3072)])
def test_mlp_residual_matches_fp32(T, D, H):
    torch.manual_seed(0)
    fc1, fc2 = nn.Linear(D, H).to(DEV).bfloat16(), nn.Linear(H, D).to(DEV).bfloat16()
    x = torch.randn(T, D, device=DEV).bfloat16()
    res = torch.randn(T, D, device=DEV).bfloat16()
    xb, rb = _leaves(x, res)
    n0 = L._STATS["xl"]
    y = L.mlp_residual(xb, rb, fc1, fc2)
    assert L._STATS["xl"] == n0 + 1, "fused path not taken"
    xf, rf, w1, b1, w2, b2 = _leaves(x.float(), res.float(), fc1.weight.float(), fc1.bias.float(),
                                     fc2.weight.float(), fc2.bias.float())
    yr = _ref_mlp(xf, rf, w1, b1, w2, b2)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(rb.grad.float(), rf.grad, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(xb.grad.float(), xf.grad, atol=0.05 * H ** 0.5 / 8, rtol=3e-2)
    torch.testing.assert_close(fc1.weight.grad.float(), w1.grad, atol=0.02 * T ** 0.5, rtol=3e-2)
    torch.testing.assert_close(fc2.weight.grad.float(), w2.grad, atol=0.02 * T ** 0.5, rtol=3e-2)
    torch.testing.assert_close(fc1.bias.grad.float(), b1.grad, atol=0.02 * T ** 0.5, rtol=3e-2)
    torch.testing.assert_close(fc2.bias.grad.float(), b2.grad, atol=0.02 * T ** 0.5, rtol=3e-2)


def test_linear_residual_matches_fp32():
    torch.manual_seed(1)
    T, D = 6000, 768
    proj = nn.Linear(D, D).to(DEV).bfloat16()
    x = torch.randn(2, T // 2, D, device=DEV).bfloat16()
    res = torch.randn(2, T // 2, D, device=DEV).bfloat16()
    xb, rb = _leaves(x, res)
    n0 = L._STATS["xl"]
    y = L.linear_residual(xb, rb, proj.weight, proj.bias)
    assert L._STATS["xl"] == n0 + 1
    xf, rf, w, b = _leaves(x.float(), res.float(), proj.weight.float(), proj.bias.float())
    yr = rf + F.linear(xf, w, b)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(rb.grad.float(), rf.grad, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(xb.grad.float(), xf.grad, atol=0.1, rtol=3e-2)
    torch.testing.assert_close(proj.weight.grad.float(), w.grad, atol=0.02 * T ** 0.5, rtol=3e-2)
    torch.testing.assert_close(proj.bias.grad.float(), b.grad, atol=0.02 * T ** 0.5, rtol=3e-2)


def test_small_token_count_uses_library_path():
    fc1, fc2 = nn.Linear(256, 1024).to(DEV).bfloat16(), nn.Linear(1024, 256).to(DEV).bfloat16()
    x = torch.randn(100, 256, device=DEV).bfloat16()
    n0 = L._STATS["xl"]
    y = L.mlp_residual(x, x, fc1, fc2)
    assert L._STATS["xl"] == n0
    torch.testing.assert_close(y.float(), (x + fc2(F.gelu(fc1(x)))).float(), atol=0.05, rtol=2e-2)


@pytest.mark.parametrize("xl", [False, True])
def test_weight_grads_on_tn_kernel_match_fp32(monkeypatch, xl):
    """Token counts past _TN_MIN_ROWS: every weight gradient of the MLP runs on
    gemm_tn_xl (split over tokens), on the library forward (linear_gelu +
    Linear) and on the fused-epilogue forward alike."""
    monkeypatch.setattr(L, "_XL", xl)
    torch.manual_seed(2)
    T, D, H = 20000, 768, 3072
    fc1, fc2 = L.Linear(D, H).to(DEV).bfloat16(), L.Linear(H, D).to(DEV).bfloat16()
    x = torch.randn(T, D, device=DEV).bfloat16()
    res = torch.randn(T, D, device=DEV).bfloat16()
    xb, rb = _leaves(x, res)
    n0 = L._STATS["tn_wgrad"]
    y = L.mlp_residual(xb, rb, fc1, fc2)
    g = torch.randn(T, D, device=DEV)
    y.backward(g.bfloat16())
    assert L._STATS["tn_wgrad"] == n0 + 2, "weight gradients did not run on gemm_tn_xl"
    xf, rf, w1, b1, w2, b2 = _leaves(x.float(), res.float(), fc1.weight.float(), fc1.bias.float(),
                                     fc2.weight.float(), fc2.bias.float())
    _ref_mlp(xf, rf, w1, b1, w2, b2).backward(g)
    for got, ref in ((fc1.weight.grad, w1.grad), (fc2.weight.grad, w2.grad)):
        err = ((got.float() - ref).norm() / ref.norm()).item()
        assert err < 2e-2, err
