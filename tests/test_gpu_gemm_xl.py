"""Large-tile transformer GEMM (csrc/gemm/gemm_xl.hip) against fp32 PyTorch
references: every epilogue (store, bias, bias+GELU with the pre-activation
side output, GELU-backward, bias+residual), both N tiles, ragged M / N tails,
K of one and many tiles, an asymmetric A = I check for a transposed C write."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def C():
    return _native.require("gemm_xl tests")


def _tol(K):
    return dict(atol=0.03 * K ** 0.5, rtol=2e-2)


@pytest.fixture(params=[(0, -1), (128, 1), (256, 1), (128, 0), (256, 0), (256, 10), (256, 11)],
                ids=["auto", "bn128", "bn256", "bn128-pipe0", "bn256-pipe0", "bn256-pingpong", "bn256-w4"])
def bn(request):
    old = C().get_gemm_xl_pipe()
    C().set_gemm_xl_bn(*request.param)
    yield request.param
    C().set_gemm_xl_bn(0, old)


@pytest.mark.parametrize("M,N,K", [(25216, 768, 768), (300, 2304, 64), (513, 136, 192), (4096, 1024, 3072),
                                   (700, 512, 128), (1100, 768, 576)])
def test_xl_store(M, N, K, bn):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    c = C().gemm_xl(a, b)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(c.float(), ref, **_tol(K))


def test_xl_identity_asymmetric(bn):
    K = 256
    a = torch.eye(K, device=DEV).bfloat16()
    b = (torch.arange(512 * K, device=DEV).reshape(512, K) % 97).bfloat16()
    c = C().gemm_xl(a, b)
    torch.testing.assert_close(c.float(), b.float().t())


@pytest.mark.parametrize("M,N,K", [(3000, 768, 768), (257, 3072, 768)])
def test_xl_bias_gelu(M, N, K, bn):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    c = C().gemm_xl(a, w, "bias", bias=bias)
    ref = F.linear(a, w, bias)  # bf16 result of the torch op
    torch.testing.assert_close(c.float(), ref.float(), atol=0.05, rtol=2e-2)
    aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    g = C().gemm_xl(a, w, "bias_gelu", bias=bias, aux=aux)
    torch.testing.assert_close(aux.float(), ref.float(), atol=0.05, rtol=2e-2)
    torch.testing.assert_close(g.float(), F.gelu(aux.float()), atol=0.02, rtol=2e-2)


def test_xl_dgelu(bn):
    torch.manual_seed(2)
    M, N, K = 1000, 3072, 768
    dy = torch.randn(M, K, device=DEV).bfloat16()
    w2t = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()  # fc2 weight^T: [hidden, dim]
    pre = torch.randn(M, N, device=DEV).bfloat16()
    c = C().gemm_xl(dy, w2t, "dgelu", aux=pre)
    dh = (dy.float() @ w2t.float().t()).bfloat16().float()
    x = pre.float().requires_grad_()
    F.gelu(x).backward(dh)
    torch.testing.assert_close(c.float(), x.grad, atol=0.05, rtol=3e-2)


def test_xl_bias_residual(bn):
    torch.manual_seed(3)
    M, N, K = 2000, 768, 3072
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    c = C().gemm_xl(a, w, "bias_res", bias=bias, residual=r)
    ref = F.linear(a, w, bias).float() + r.float()
    torch.testing.assert_close(c.float(), ref, atol=0.06, rtol=2e-2)


def test_xl_strided_operands_and_out():
    torch.manual_seed(4)
    big = torch.randn(700, 3 * 256, device=DEV).bfloat16()
    a = big[:, 256:512]  # row stride 768
    b = (torch.randn(384, 256, device=DEV) * 0.1).bfloat16()
    out = torch.empty(700, 2 * 384, device=DEV, dtype=torch.bfloat16)
    C().gemm_xl(a, b, out=out[:, 384:])
    torch.testing.assert_close(out[:, 384:].float(), a.float() @ b.float().t(), **_tol(256))


def test_xl_rejects_bad_k():
    a = torch.randn(64, 100, device=DEV).bfloat16()
    b = torch.randn(64, 100, device=DEV).bfloat16()
    with pytest.raises(RuntimeError):
        C().gemm_xl(a, b)
