"""Native LayerNorm (one wave per row) vs an fp32 F.layer_norm reference."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.layernorm import _STATS, layer_norm

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype,pdtype", [(torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
                                          (torch.float32, torch.float32)])
@pytest.mark.parametrize("shape", [(128, 197, 768), (3, 5, 768), (7, 1024), (3, 5, 1536), (2, 2048), (1000, 64)])
def test_layernorm_fwd_bwd(dtype, pdtype, shape):
    torch.manual_seed(0)
    d = shape[-1]
    x = (torch.randn(*shape, device="cuda") * 2 + 0.5).to(dtype)
    w = (torch.rand(d, device="cuda") + 0.5).to(pdtype).requires_grad_()
    b = torch.randn(d, device="cuda").to(pdtype).requires_grad_()
    xi = x.detach().requires_grad_()
    n0 = _STATS["native"]
    y = layer_norm(xi, (d,), w, b, 1e-6)
    assert _STATS["native"] == n0 + 1
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_()
    yr = F.layer_norm(xr, (d,), wr, br, 1e-6)
    tol = 3e-2 if dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=tol * 2, rtol=tol)
    rows = x.numel() // d
    gtol = (2e-2 if pdtype == torch.bfloat16 else 1e-3) * rows ** 0.5
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=gtol, rtol=2e-2)
    torch.testing.assert_close(b.grad.float(), br.grad, atol=gtol, rtol=2e-2)


def test_vit_block_residual_grad_fused_into_layernorm():
    """Pre-LN block: each LayerNorm's backward absorbs the residual branch's gradient
    (GradSlot); x.grad must match the plain composition of the same modules."""
    import copy
    from distributed_model_parallel_amd.models.vit import EncoderBlock
    torch.manual_seed(0)
    blk = EncoderBlock(768, 12, 3072).cuda().bfloat16().train()
    ref = copy.deepcopy(blk)
    x = torch.randn(4, 197, 768, device="cuda").bfloat16()
    xa, xb = x.detach().requires_grad_(), x.detach().requires_grad_()
    n0 = _STATS["fused_residual_grad"]
    ya = blk(xa)
    h = xb + ref.attn(ref.ln1(xb))
    yb = h + ref.mlp(ref.ln2(h))
    torch.testing.assert_close(ya.float(), yb.float(), atol=2e-2, rtol=2e-2)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    assert _STATS["fused_residual_grad"] == n0 + 2
    err = (xa.grad.float() - xb.grad.float()).norm() / xb.grad.float().norm()
    assert err < 2e-2, err


@pytest.mark.parametrize("has_w,has_b", [(False, False), (True, False), (False, True)])
def test_layernorm_absent_affine(has_w, has_b):
    """An absent weight / bias reaches the kernel as ones / zeros."""
    torch.manual_seed(0)
    d = 768
    x = torch.randn(6, 33, d, device="cuda").bfloat16()
    w = (torch.rand(d, device="cuda") + 0.5).requires_grad_() if has_w else None
    b = torch.randn(d, device="cuda").requires_grad_() if has_b else None
    xi = x.detach().requires_grad_()
    y = layer_norm(xi, (d,), w, b, 1e-5)
    xr = x.detach().float().requires_grad_()
    yr = F.layer_norm(xr, (d,), w, None, 1e-5)  # stock ROCm backward rejects (None, bias)
    if has_b:
        yr = yr + b
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=3e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    wg = w.grad.clone() if has_w else None
    if has_w:
        w.grad = None
    if has_b:
        bg = b.grad.clone()
        b.grad = None
    yr.backward(g.bfloat16().float())
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=6e-2, rtol=3e-2)
    if has_w:
        torch.testing.assert_close(wg, w.grad, atol=0.5, rtol=2e-2)
    if has_b:
        torch.testing.assert_close(bg, b.grad, atol=0.5, rtol=2e-2)
