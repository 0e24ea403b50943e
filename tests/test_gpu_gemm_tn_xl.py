"""Weight-gradient GEMM on the ping-pong schedule (csrc/gemm/gemm_xl.hip
gemm_tn_pp_kernel: m-major LDS planes, transposing LDS reads, split over M)
against fp32 torch: plain A^T B with ragged M / N / K, and the implicit-GEMM
conv weight gradient (3x3, strided, 1x1 strided) against autograd."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


@pytest.mark.parametrize("M,N,K", [(802816 // 4, 256, 1024), (5000, 200, 264), (100, 256, 256), (64, 512, 512),
                                   (33, 64, 128), (50176, 2048, 512)])
@pytest.mark.parametrize("out", [torch.float32, torch.bfloat16])
def test_gemm_tn_xl(M, N, K, out):
    C = _native.require("gemm_tn_xl")
    torch.manual_seed(0)
    a = torch.randn(M, N, device=DEV).bfloat16()
    b = torch.randn(M, K, device=DEV).bfloat16()
    got = C.gemm_tn_xl(a, b, out)
    ref = a.float().t() @ b.float()
    tol = 1e-3 * M ** 0.5 + (0.02 * ref.abs().max().item() if out == torch.bfloat16 else 0)
    torch.testing.assert_close(got.float(), ref, atol=tol, rtol=1e-2)


@pytest.mark.parametrize("M", [640, 64, 192, 320, 576])
def test_gemm_tn_xl_exact_pattern(M):
    """Exact small-integer products; M = 64..576 covers 1..9 K tiles per split
    (fewer than the ring's 9-unit prologue and the tail of the counted waits)."""
    C = _native.require("gemm_tn_xl")
    N, K = 256, 512
    a = (torch.arange(M * N, device=DEV).reshape(M, N) % 7 - 3).bfloat16()
    b = (torch.arange(M * K, device=DEV).reshape(M, K) % 5 - 2).bfloat16()
    assert torch.equal(C.gemm_tn_xl(a, b, torch.float32), a.float().t() @ b.float())


@pytest.fixture(params=[10, 11])
def tn_pipe(request):
    """10: the ping-pong TN kernel; 11: the 4-wave one (its tap gather walks
    each staged row's pixel forward 64 at a time: ho 5 / 7 exercise the
    multi-image wrap, ho 3 falls back to the ping-pong kernel)."""
    C = _native.require("conv_wgrad_xl")
    old = C.get_gemm_xl_pipe()
    C.set_gemm_xl_bn(0, request.param, 0)
    yield request.param
    C.set_gemm_xl_bn(0, old, 0)


@pytest.mark.parametrize("n,cin,cout,h,k,s", [(4, 256, 256, 9, 3, 1), (3, 256, 512, 15, 3, 2), (2, 512, 256, 7, 3, 1),
                                              (4, 256, 128, 10, 1, 2), (64, 512, 512, 7, 3, 1),
                                              (24, 256, 256, 14, 3, 2), (9, 256, 256, 5, 3, 1), (16, 256, 256, 3, 3, 1)])
def test_conv_wgrad_xl(n, cin, cout, h, k, s, tn_pipe):
    C = _native.require("conv_wgrad_xl")
    torch.manual_seed(1)
    p = k // 2
    ho = (h + 2 * p - k) // s + 1
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    dy = torch.randn(n, cout, ho, ho, device=DEV).bfloat16().contiguous(memory_format=CL)
    dy2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
    got = C.conv_wgrad_xl(dy2, x, k, k, s, p, ho, ho, torch.float32).view(cout, k, k, cin).permute(0, 3, 1, 2)
    wr = torch.zeros(cout, cin, k, k, device=DEV, requires_grad=True)
    F.conv2d(x.float(), wr, None, s, p).backward(dy.float())
    torch.testing.assert_close(got, wr.grad, atol=2e-3 * (n * ho * ho) ** 0.5, rtol=1e-2)


@pytest.mark.parametrize("n,cin,h,s", [(8, 256, 28, 2), (32, 512, 14, 2), (16, 1024, 14, 2), (8, 256, 9, 2)])
def test_gram_strided_xl(n, cin, h, s):
    """Gram of a strided 1x1 sample with both operands gathered in place
    (gemm_tn_w4_kernel<3>) against the fp32 Gram of the sliced sample."""
    C = _native.require("gram_strided_xl")
    torch.manual_seed(2)
    ho = (h - 1) // s + 1
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    assert C.gram_strided_xl_supported(n, cin, h, h, ho, ho)
    got = C.gram_strided_xl(x, s, ho, ho)
    xs = x[:, :, ::s, ::s].permute(0, 2, 3, 1).reshape(-1, cin).float()
    ref = xs.t() @ xs
    torch.testing.assert_close(got, ref, atol=2e-3 * (n * ho * ho) ** 0.5, rtol=1e-3)


def test_strided_gather_over_2gb_input():
    """ResNet-50 layer-2 downsample at batch 2048: the 3.3 GB NHWC input is
    past 32-bit offsets from its start; each M split addresses it from its
    own first image.  Weight gradient and Gram against fp32 references on a
    sub-sample of the output channels."""
    C = _native.require("conv_wgrad_xl")
    torch.manual_seed(3)
    n, cin, h, cout = 2048, 256, 56, 256
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    assert x.numel() * 2 > 2 ** 31
    ho = h // 2
    xs = x[:, :, ::2, ::2].permute(0, 2, 3, 1).reshape(-1, cin)
    dy2 = torch.randn(n * ho * ho, cout, device=DEV).bfloat16()
    got = C.conv_wgrad_xl(dy2, x, 1, 1, 2, 0, ho, ho, torch.float32)
    ref = dy2.float().t() @ xs.float()
    torch.testing.assert_close(got, ref, atol=3e-3 * (n * ho * ho) ** 0.5, rtol=1e-3)
    assert C.gram_strided_xl_supported(n, cin, h, h, ho, ho)
    g = C.gram_strided_xl(x, 2, ho, ho)
    gr = xs.float().t() @ xs.float()
    torch.testing.assert_close(g, gr, atol=3e-3 * (n * ho * ho) ** 0.5, rtol=1e-3)


@pytest.mark.parametrize("M,N,K", [(200000, 64, 256), (200000, 256, 64), (100000, 128, 512), (100000, 512, 128),
                                   (70000, 64, 64), (5000, 64, 320), (3000, 200, 120), (4133, 128, 256),
                                   (64, 64, 256), (40000, 24, 144), (40000, 144, 24), (33000, 16, 96),
                                   (20000, 32, 32)])
@pytest.mark.parametrize("narrow", [True, False])
def test_gemm_tn_xl_narrow_tiles(M, N, K, narrow):
    """The 4-wave weight-gradient kernel's narrow tiles (64 x 256, 256 x 64,
    128 x 256, 256 x 128: gemm_tn_w4_kernel<0, TNN, TNK>) against fp32, with
    the accumulate-into-out path; narrow=False: the 256 x 256 tile."""
    C = _native.require("gemm_tn_xl")
    C.set_tn_narrow(narrow)
    try:
        torch.manual_seed(11)
        a = torch.randn(M, N, device=DEV).bfloat16()
        b = torch.randn(M, K, device=DEV).bfloat16()
        ref = a.float().t() @ b.float()
        got = C.gemm_tn_xl(a, b, torch.float32)
        torch.testing.assert_close(got, ref, atol=1e-3 * M ** 0.5, rtol=1e-2)
        acc = torch.randn(N, K, device=DEV)
        acc0 = acc.clone()
        C.gemm_tn_xl(a, b, torch.float32, out=acc)
        torch.testing.assert_close(acc, acc0 + ref, atol=1e-3 * M ** 0.5, rtol=1e-2)
    finally:
        C.set_tn_narrow(True)
