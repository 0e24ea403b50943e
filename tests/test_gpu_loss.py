"""Fused cross-entropy HIP kernels vs F.cross_entropy in fp32."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.loss import _STATS, cross_entropy

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C", [(1024, 1000), (7, 10), (33, 365), (5, 70)])
def test_cross_entropy_matches_torch(dtype, B, C):
    torch.manual_seed(0)
    x = (torch.randn(B, C, device="cuda") * 3).to(dtype)
    t = torch.randint(0, C, (B,), device="cuda")
    t[0] = -100  # ignored row
    xa = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    n0 = _STATS["native"]
    la = cross_entropy(xa, t)
    assert _STATS["native"] == n0 + 1
    lr = F.cross_entropy(xr, t)
    torch.testing.assert_close(la, lr, atol=1e-5, rtol=1e-5)
    (la * 2.0).backward()
    (lr * 2.0).backward()
    tol = 1e-6 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(xa.grad.float(), xr.grad, atol=tol, rtol=1e-2)
    assert xa.grad.dtype == dtype


@pytest.mark.parametrize("bad", [10, 12345, -3])
def test_cross_entropy_out_of_range_label_is_nan_not_oob(bad):
    """a label outside [0, C) must not read past the row (the fused
    kernel replaces F.cross_entropy, which raises); it poisons loss and grad."""
    x = torch.randn(8, 10, device="cuda", requires_grad=True)
    t = torch.randint(0, 10, (8,), device="cuda")
    t[3] = bad
    loss = cross_entropy(x, t)
    assert torch.isnan(loss).item()
    loss.backward()
    assert torch.isnan(x.grad[3]).all().item()


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,C", [(64, 10), (33, 4), (256, 1000)])
def test_cross_entropy_with_stats_matches_topk(dtype, B, C):
    """The pipeline's fused loss + statistics (ops/loss.py cross_entropy_with_stats):
    scale * loss, its gradient, and stats += (loss, top-1, top-min(5,C) correct)
    against F.cross_entropy and torch.topk (bf16 logits: ties between equal
    logits resolved by index, as a stable sort)."""
    from distributed_model_parallel_amd.ops.loss import cross_entropy_with_stats
    torch.manual_seed(B + C)
    x = (torch.randn(B, C, device="cuda") * 3).to(dtype)
    t = torch.randint(0, C, (B,), device="cuda")
    stats = torch.full((3,), 1.5, dtype=torch.float64, device="cuda")  # accumulates
    xa = x.clone().requires_grad_()
    loss = cross_entropy_with_stats(xa, t, 0.25, stats)
    loss.backward()
    xr = x.float().clone().requires_grad_()
    ref = F.cross_entropy(xr, t) * 0.25
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    torch.testing.assert_close(xa.grad.float(), xr.grad, atol=1e-2 if dtype == torch.bfloat16 else 1e-6, rtol=1e-2)
    k = min(5, C)
    xf = x.float()
    xt = xf.gather(1, t[:, None])
    idx = torch.arange(C, device="cuda")[None, :]
    rank = ((xf > xt) | ((xf == xt) & (idx < t[:, None]))).sum(1)
    assert abs(float(stats[0]) - 1.5 - float(ref)) < 1e-5 * max(1.0, abs(float(ref)))
    assert float(stats[1]) - 1.5 == float((rank < 1).sum())
    assert float(stats[2]) - 1.5 == float((rank < k).sum())
    if dtype == torch.float32:  # no ties: the same counts as torch.topk
        top = xf.topk(k, 1).indices
        assert float(stats[1]) - 1.5 == float((top[:, 0] == t).sum())
        assert float(stats[2]) - 1.5 == float((top == t[:, None]).any(1).sum())
