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


@pytest.mark.parametrize("T", [50432, 1000])
def test_dgelu_epilogue_bias_grad(T):
    """fc1's bias gradient as column sums from fc2's data-gradient epilogue
    (gemm_xl_dgelu_bgrad) vs an fp32 reference of the same math."""
    from distributed_model_parallel_amd import _native
    C = _native.require("test")
    torch.manual_seed(3)
    D, H = 768, 3072
    dy = torch.randn(T, D, device=DEV).bfloat16()
    w2t = (torch.randn(H, D, device=DEV) * 0.05).bfloat16()
    h = torch.randn(T, H, device=DEV).bfloat16()
    dh, db = C.gemm_xl_dgelu_bgrad(dy, w2t, h)
    assert torch.equal(dh, C.gemm_xl(dy, w2t, "dgelu", aux=h))
    torch.testing.assert_close(db, dh.float().sum(0), atol=1e-2 * T ** 0.5, rtol=1e-4)
    hf = h.float()
    ref = (dy.float() @ w2t.float().t()) * (0.5 * (1 + torch.erf(hf / 2 ** 0.5)) +
                                             hf * torch.exp(-0.5 * hf * hf) / (2 * torch.pi) ** 0.5)
    assert ((db - ref.sum(0)).norm() / ref.sum(0).norm()).item() < 1e-2


@pytest.mark.parametrize("mode", ["xl", "fwd", "lib"])
def test_qkv_linear_forward_and_dgrad_on_xl(mode, monkeypatch):
    """The qkv projection (ops.linear.linear -> _LinearFn): forward with the
    bias in gemm_xl's store and the data gradient on gemm_xl
    (DMP_LINEAR_PLAIN=xl, the default), the forward only ("fwd"), or both on
    hipBLASLt ("lib")."""
    monkeypatch.setattr(L, "_PLAIN_FWD_XL", mode in ("xl", "fwd"))
    monkeypatch.setattr(L, "_PLAIN_DGRAD_XL", mode == "xl")
    torch.manual_seed(4)
    T, D = 8192, 768
    qkv = nn.Linear(D, 3 * D).to(DEV).bfloat16()
    x = torch.randn(T, D, device=DEV).bfloat16()
    (xb,) = _leaves(x)
    f0, d0 = L._STATS["xl_fwd"], L._STATS["xl_dgrad"]
    y = L.linear(xb, qkv.weight, qkv.bias)
    assert L._STATS["xl_fwd"] == f0 + (1 if mode in ("xl", "fwd") else 0)
    xf, w, b = _leaves(x.float(), qkv.weight.float(), qkv.bias.float())
    yr = F.linear(xf, w, b)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    assert L._STATS["xl_dgrad"] == d0 + (1 if mode == "xl" else 0)
    torch.testing.assert_close(xb.grad.float(), xf.grad, atol=0.05 * (3 * D) ** 0.5 / 8, rtol=3e-2)
    err = ((qkv.weight.grad.float() - w.grad).norm() / w.grad.norm()).item()
    assert err < 2e-2, err


@pytest.mark.parametrize("B", [32, 3])
def test_patch_embed_gemm_matches_conv(B):
    """16x16/s16 patch embedding as one GEMM (ops/patch_embed.py) vs the fp32
    convolution: tokens, weight and bias gradients (B = 3: 588 rows -> torch path)."""
    from distributed_model_parallel_amd.ops import patch_embed as P
    torch.manual_seed(5)
    pe = P.PatchEmbed(3, 768, 16).to(DEV).bfloat16().to(memory_format=torch.channels_last)
    x = torch.randn(B, 3, 224, 224, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    n0 = P._STATS["native"]
    y = pe(x)
    assert y.shape == (B, 196, 768)
    if B * 196 >= L._XL_MIN_ROWS:
        assert P._STATS["native"] == n0 + 1
    w, b = _leaves(pe.weight.float(), pe.bias.float())
    yr = F.conv2d(x.float(), w, b, stride=16).flatten(2).transpose(1, 2)
    torch.testing.assert_close(y.float(), yr, atol=0.05, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    err = ((pe.weight.grad.float() - w.grad).norm() / w.grad.norm()).item()
    assert err < 2e-2, err
    torch.testing.assert_close(pe.bias.grad.float(), b.grad, atol=0.02 * (B * 196) ** 0.5, rtol=3e-2)
