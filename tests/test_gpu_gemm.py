"""MFMA GEMM (csrc/conv/gemm_bf16.hip) against an fp32 PyTorch reference:
plain, BN-moments epilogue, BN-apply+ReLU prologue, eval-mode affine(+res)+ReLU
epilogue; odd M, ragged K tiles, every N-tile variant; an asymmetric operand
check (A = I) that catches a transposed C write."""
import pytest
import torch

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"


def C():
    return _native.require("gemm tests")


def _ref(a, b, s=None, t=None):
    a = a.float()
    if s is not None:
        a = torch.relu(a * s + t)
        a = a.bfloat16().float()  # the kernel stages the prologue output as bf16
    return a @ b.float().t()


@pytest.mark.parametrize("M,N,K", [(1000, 64, 256), (4097, 128, 64), (333, 256, 24), (2048, 2048, 512),
                                   (127, 8, 8), (50176, 64, 64)])
def test_gemm_store(M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    c, mom = C().gemm_nt(a, b)
    assert mom is None or not mom.numel()
    ref = _ref(a, b)
    torch.testing.assert_close(c.float(), ref, atol=0.05 * K ** 0.5, rtol=2e-2)


def test_gemm_identity_asymmetric():
    K = 64
    a = torch.eye(K, device=DEV).bfloat16()
    b = (torch.arange(128 * K, device=DEV).reshape(128, K) % 97).bfloat16()
    c, _ = C().gemm_nt(a, b)
    torch.testing.assert_close(c.float(), b.float().t())


@pytest.mark.parametrize("M,N,K", [(3000, 64, 256), (777, 256, 64)])
def test_gemm_moments(M, N, K):
    torch.manual_seed(1)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    c, mom = C().gemm_nt(a, b, mode="moments")
    cf = c.float().double()
    torch.testing.assert_close(mom[:N], cf.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(mom[N:2 * N], (cf * cf).sum(0), atol=1e-2, rtol=1e-4)
    assert mom[2 * N].item() == M


@pytest.mark.parametrize("M,N,K", [(1500, 128, 128), (640, 64, 72)])
def test_gemm_bn_prologue(M, N, K):
    torch.manual_seed(2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    s = torch.rand(K, device=DEV) + 0.5
    t = torch.randn(K, device=DEV)
    c, _ = C().gemm_nt(a, b, s, t)
    torch.testing.assert_close(c.float(), _ref(a, b, s, t), atol=0.05 * K ** 0.5, rtol=2e-2)


@pytest.mark.parametrize("res", [False, True])
def test_gemm_affine_epilogue(res):
    torch.manual_seed(3)
    M, N, K = 999, 256, 64
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    es = torch.rand(N, device=DEV)
    et = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).bfloat16() if res else None
    c, _ = C().gemm_nt(a, b, mode="affine", epi_scale=es, epi_shift=et, residual=r, relu=True)
    ref = _ref(a, b).bfloat16().float() * es + et
    if res:
        ref = ref + r.float()
    torch.testing.assert_close(c.float(), torch.relu(ref), atol=0.05 * K ** 0.5, rtol=2e-2)


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5, 6])
@pytest.mark.parametrize("mode", ["store", "moments"])
def test_gemm_tile_variants(tile, mode):
    """Every NT tile variant (set_gemm_tile) against fp32, incl. the 8-wave 256x128 one."""
    c = C()
    torch.manual_seed(tile)
    M, N, K = 1000, 192, 320
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = torch.randn(N, K, device=DEV).bfloat16()
    c.set_gemm_tile(tile)
    try:
        y, mom = c.gemm_nt(a, b, mode=mode)
    finally:
        c.set_gemm_tile(-1)
    ref = a.float() @ b.float().t()
    torch.testing.assert_close(y.float(), ref, atol=0.05 * K ** 0.5, rtol=2e-2)
    if mode == "moments":
        yf = y.float()
        torch.testing.assert_close(mom[:N].float(), yf.sum(0), atol=1e-2 * M ** 0.5, rtol=1e-3)
