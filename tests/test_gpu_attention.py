"""Fused packed-qkv attention (csrc/attn/attention.hip) against an fp32
PyTorch reference: forward output, and dq/dk/dv through the packed dqkv
gradient, at ViT-B/16's S = 197 and at other padded lengths (S = 1, 17, 64,
130, 256); plus the ViT block path using it."""
import math

import pytest
import torch

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops import attention as A

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(qkv, heads):
    b, s, d3 = qkv.shape
    d = d3 // 3
    hd = d // heads
    q, k, v = qkv.float().view(b, s, 3, heads, hd).permute(2, 0, 3, 1, 4).unbind(0)
    att = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    o = att.softmax(-1) @ v
    return o.transpose(1, 2).reshape(b, s, d)


@pytest.mark.parametrize("B,S,H", [(4, 197, 12), (3, 1, 2), (2, 17, 3), (2, 64, 4), (2, 130, 2), (1, 256, 2)])
def test_attention_fwd_bwd(B, S, H):
    _native.require("attention test")
    torch.manual_seed(0)
    d = H * 64
    qkv = (torch.randn(B, S, 3 * d, device=DEV) * 1.5).bfloat16().requires_grad_()
    o = A.self_attention_packed(qkv, H)
    assert A._STATS["native"] > 0
    ref_in = qkv.detach().float().requires_grad_()
    ref = _ref(ref_in, H)
    torch.testing.assert_close(o.float(), ref, atol=2e-2, rtol=2e-2)
    go = torch.randn_like(ref)
    o.backward(go.bfloat16())
    ref.backward(go)
    g, gr = qkv.grad.float(), ref_in.grad
    # per-part relative error (q, k, v blocks)
    for i in range(3):
        a, r = g[..., i * d:(i + 1) * d], gr[..., i * d:(i + 1) * d]
        # S = 1: dq = dk = 0 exactly in theory (softmax of one key), so bound
        # the error relative to the whole gradient as well
        err = (a - r).norm().item()
        assert err <= 2e-2 * r.norm().item() + 1e-3 * gr.norm().item(), (i, err, r.norm().item())


def test_attention_matches_sdpa_path_in_vit_block():
    from distributed_model_parallel_amd.models.vit import EncoderBlock
    torch.manual_seed(1)
    blk = EncoderBlock(768, 12, 3072).to(DEV).bfloat16()
    x = torch.randn(2, 197, 768, device=DEV).bfloat16()
    y = blk(x)
    with torch.no_grad():
        h = blk.ln1(x)
        qkv = blk.attn.qkv(h)
        ref = blk.attn.proj(_ref(qkv, 12).bfloat16())
    got = blk.attn(h)
    torch.testing.assert_close(got.float(), ref.float(), atol=3e-2, rtol=3e-2)
    assert torch.isfinite(y).all()


def test_attention_variants_agree_bitwise():
    """The persistent forward (next-head K / V / Q prefetch) computes exactly
    what the one-workgroup-per-head kernel computes (same MFMA order)."""
    from distributed_model_parallel_amd import _native
    C = _native.require("attention")
    torch.manual_seed(9)
    B, S, H = 40, 197, 12  # 480 heads: fewer and more than 2 x CUs per wave of the grid
    qkv = torch.randn(B * S, 3 * H * 64, device="cuda").bfloat16()
    do = torch.randn(B * S, H * 64, device="cuda").bfloat16()
    try:
        C.set_attention_variant(0, 0)
        o0, l0 = C.attention_forward(qkv, B, S, H, 0.125)
        g0 = C.attention_backward(do, qkv, o0, l0, B, S, H, 0.125)
        C.set_attention_variant(1, 1)
        o1, l1 = C.attention_forward(qkv, B, S, H, 0.125)
        g1 = C.attention_backward(do, qkv, o0, l0, B, S, H, 0.125)
        C.set_attention_variant(2, 1)
        o2, l2 = C.attention_forward(qkv, B, S, H, 0.125)
        C.set_attention_variant(3, 0)
        o3, l3 = C.attention_forward(qkv, B, S, H, 0.125)
    finally:
        C.set_attention_variant(0, 0)
    assert torch.equal(o0, o1) and torch.equal(o0, o2) and torch.equal(o0, o3)
    assert torch.equal(l0[:, :S], l1[:, :S]) and torch.equal(l0[:, :S], l2[:, :S]) and torch.equal(l0[:, :S], l3[:, :S])
    assert torch.equal(g0, g1), "persistent backward differs from the per-head backward"


@pytest.mark.parametrize("fv,bv", [(0, 0), (1, 1), (2, 0), (3, 0)])
@pytest.mark.parametrize("B,S,H", [(4, 197, 12), (2, 17, 3), (2, 130, 2), (1, 256, 2)])
def test_attention_variant_numerics(fv, bv, B, S, H):
    """Every forward / backward variant against the fp32 reference, at padded
    and unpadded lengths (the key-padding masks differ per variant)."""
    C = _native.require("attention")
    old = C.get_attention_variant()
    try:
        C.set_attention_variant(fv, bv)
        test_attention_fwd_bwd(B, S, H)
    finally:
        C.set_attention_variant(*old)
