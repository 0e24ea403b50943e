"""Split-M MFMA weight-gradient GEMM (transposing LDS reads) vs fp32 torch,
and the full native 1x1-conv autograd path vs F.conv2d."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops.conv1x1 import _STATS, Conv1x1

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(802816, 256, 64), (5000, 64, 256), (777, 128, 128), (64, 64, 64),
                                   (12544, 2048, 512), (100, 24, 144), (33, 8, 16)])
@pytest.mark.parametrize("out", [torch.float32, torch.bfloat16])
def test_gemm_tn(M, N, K, out):
    C = _native.require("gemm_tn")
    torch.manual_seed(0)
    a = torch.randn(M, N, device=DEV).bfloat16()
    b = torch.randn(M, K, device=DEV).bfloat16()
    got = C.gemm_tn(a, b, out)
    ref = a.float().t() @ b.float()
    tol = 1e-3 * M ** 0.5 + (0.02 * ref.abs().max().item() if out == torch.bfloat16 else 0)
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=1e-2)


def test_gemm_tn_asymmetric_pattern():
    """Exact small-integer data: any transpose/mapping slip changes the result."""
    C = _native.require("gemm_tn")
    M, N, K = 96, 64, 80
    a = (torch.arange(M * N, device=DEV).reshape(M, N) % 7 - 3).bfloat16()
    b = (torch.arange(M * K, device=DEV).reshape(M, K) % 5 - 2).bfloat16()
    torch.testing.assert_close(C.gemm_tn(a, b, torch.float32), a.float().t() @ b.float())


@pytest.mark.parametrize("stride", [1, 2])
def test_conv1x1_autograd_matches_conv2d(stride):
    torch.manual_seed(1)
    m = Conv1x1(64, 128, stride).cuda().bfloat16()
    x = torch.randn(4, 64, 14, 14, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    xi = x.detach().requires_grad_()
    n0 = _STATS["native"]
    y = m(xi)
    assert _STATS["native"] == n0 + 1
    yr = F.conv2d(xr, wr, None, stride)
    torch.testing.assert_close(y.float(), yr, atol=0.1, rtol=2e-2)
    g = torch.randn_like(yr)
    y.backward(g.bfloat16())
    yr.backward(g)
    torch.testing.assert_close(xi.grad.float(), xr.grad, atol=0.1, rtol=2e-2)
    torch.testing.assert_close(m.weight.grad.float(), wr.grad, atol=0.5, rtol=2e-2)
