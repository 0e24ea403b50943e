"""NHWC max pooling (byte argmax, gather backward) vs F.max_pool2d."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.pool import _STATS, max_pool2d

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("shape,k,s,p", [((2, 64, 112, 112), 3, 2, 1), ((3, 16, 9, 7), 3, 2, 1),
                                         ((2, 8, 10, 10), 2, 2, 0), ((1, 32, 11, 13), 3, 1, 1),
                                         ((2, 24, 8, 8), 5, 3, 2)])
def test_maxpool_matches_torch(dtype, shape, k, s, p):
    torch.manual_seed(0)
    # distinct values per window so argmax ties cannot differ in tie-breaking
    x = torch.randn(*shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    n0 = _STATS["native"]
    y = max_pool2d(xi, k, s, p)
    assert _STATS["native"] == n0 + 1
    yr = F.max_pool2d(xr, k, s, p)
    torch.testing.assert_close(y.float(), yr)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-6
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=tol, rtol=tol)


def test_maxpool_ties_first_wins():
    x = torch.zeros(1, 8, 4, 4, device="cuda").contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    xr = x.detach().requires_grad_()
    max_pool2d(xi, 2, 2, 0).sum().backward()
    F.max_pool2d(xr, 2, 2, 0).sum().backward()
    torch.testing.assert_close(xi.grad, xr.grad)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_maxpool_k3s2_fixed_path_ties_and_borders(dtype):
    """The k=3/s=2 fast path loads clamped taps unconditionally: all-equal
    inputs (every window a tie) and odd sizes check the masking at the borders
    and PyTorch's first-maximum tie-breaking."""
    x = torch.zeros(2, 16, 7, 9, device="cuda", dtype=dtype).contiguous(memory_format=torch.channels_last)
    x[1, :, 3:, :4] = 1.0
    xi = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    y = max_pool2d(xi, 3, 2, 1)
    yr = F.max_pool2d(xr, 3, 2, 1)
    torch.testing.assert_close(y.float(), yr)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-6
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=tol, rtol=tol)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_global_avg_pool_matches_torch(dtype):
    from distributed_model_parallel_amd.ops.pool import global_avg_pool
    torch.manual_seed(0)
    x = torch.randn(4, 64, 7, 5, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    xr = x.detach().float().requires_grad_()
    n0 = _STATS["native_gap"]
    y = global_avg_pool(xi)
    assert _STATS["native_gap"] == n0 + 1
    yr = torch.flatten(F.adaptive_avg_pool2d(xr, 1), 1)
    tol = 1e-2 if dtype == torch.bfloat16 else 1e-5
    torch.testing.assert_close(y.float(), yr, atol=tol, rtol=tol)
    g = torch.randn_like(yr)
    y.backward(g.to(dtype))
    yr.backward(g.to(dtype).float())
    assert xi.grad.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=tol, rtol=tol)


@pytest.mark.parametrize("k,s,p", [(3, 2, 1), (3, 1, 1)])
def test_maxpool_all_neg_inf_border_window(k, s, p):
    # every value -inf: each window's gradient must land on its first in-bounds
    # pixel -- PyTorch's CPU / NCHW semantics (its GPU NHWC kernel instead routes
    # every such window to absolute index 0), not on a padding tap that the
    # backward can never match (the gradient would be dropped)
    x = torch.full((1, 8, 6, 6), float("-inf"), device="cuda").contiguous(memory_format=torch.channels_last)
    xi = x.detach().requires_grad_()
    xr = x.detach().cpu().contiguous().requires_grad_()
    max_pool2d(xi, k, s, p).sum().backward()
    F.max_pool2d(xr, k, s, p).sum().backward()
    torch.testing.assert_close(xi.grad.cpu(), xr.grad)
