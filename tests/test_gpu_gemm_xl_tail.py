"""Split-K tail of the 256x256 ping-pong GEMMs (csrc/gemm/gemm_xl.hip
launch_pp256, DMP_XL_TAIL / set_gemm_xl_tail, off by default: the last,
partly filled round of tiles runs with its K split over
the idle CUs, fp32 partials summed by gemm_xl_tail_epi, which then runs the
tile's epilogue).  Every epilogue the split serves, on grids that trigger it
(a few tiles past a full round, and a grid smaller than half the chip), against
the same call with the split off and against fp32 references: only the fp32
summation order differs."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


@pytest.fixture
def C():
    c = _native.require("gemm_xl tail tests")
    old = c.get_gemm_xl_tail()
    yield c
    c.set_gemm_xl_tail(old)


def both(C, fn):
    C.set_gemm_xl_tail(0)
    ref = fn()
    C.set_gemm_xl_tail(1)
    out = fn()
    torch.cuda.synchronize()
    return ref, out


def wmat(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


# n images of h x h: 1356 x 49 = 66444 rows = 260 M tiles (4 past a full
# round of 256 CUs); 200 x 49 = 9800 rows x 2 N tiles = 78 tiles (< half)
@pytest.mark.parametrize("n,cin,cout,h", [(1356, 256, 256, 7), (200, 512, 512, 7), (6, 256, 256, 14)])
def test_conv_xl_tail_moments(C, n, cin, cout, h):
    torch.manual_seed(0)
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.05).bfloat16()
    (y0, s0), (y1, s1) = both(C, lambda: C.conv_xl(x, wmat(w), 3, 3, 1, 1, h, h, "moments"))
    torch.testing.assert_close(y1.float(), y0.float(), atol=3e-2, rtol=1e-2)
    rows = n * h * h
    torch.testing.assert_close(s1[:2 * cout], s0[:2 * cout], atol=2e-2 * rows ** 0.5, rtol=1e-3)
    assert s1[2 * cout].item() == rows
    if n <= 200:
        ref = F.conv2d(x.float(), w.float(), None, 1, 1).permute(0, 2, 3, 1).reshape(-1, cout)
        torch.testing.assert_close(y1.float(), ref, atol=5e-2, rtol=2e-2)


def test_conv_xl_tail_bnbwd_and_add(C):
    torch.manual_seed(1)
    n, c, h = 1356, 256, 7
    rows = n * h * h
    dy = torch.randn(n, c, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = (torch.randn(c, c * 9, device=DEV) * 0.05).bfloat16()
    x = torch.randn(rows, c, device=DEV).bfloat16()
    res = torch.randn(rows, c, device=DEV).bfloat16()
    mean = torch.randn(c, device=DEV) * 0.1
    inv = torch.rand(c, device=DEV) + 0.5
    bw = torch.rand(c, device=DEV) + 0.5
    bb = torch.randn(c, device=DEV) * 0.1
    (g0, t0), (g1, t1) = both(C, lambda: C.conv_xl(dy, w, 3, 3, 1, 1, h, h, "bnbwd", bn_x=x, mean=mean, invstd=inv,
                                                   weight=bw, bias=bb))
    torch.testing.assert_close(g1.float(), g0.float(), atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(t1[:2 * c], t0[:2 * c], atol=2e-2 * rows ** 0.5, rtol=1e-3)
    (a0, _), (a1, _) = both(C, lambda: C.conv_xl(dy, w, 3, 3, 1, 1, h, h, "add", residual=res))
    torch.testing.assert_close(a1.float(), a0.float(), atol=3e-2, rtol=1e-2)


def test_gemm_xl_conv_tail_fold_dgrad(C):
    """The folded dgrad (two-source A, ebias, BN backward) at K = 1280: 257 tiles."""
    torch.manual_seed(2)
    w, rows = 256, 257 * 256 - 5
    dz = torch.randn(rows, 4 * w, device=DEV).bfloat16()
    a = torch.randn(rows, w, device=DEV).bfloat16()
    Bb = (torch.randn(w, 5 * w, device=DEV) * 0.03).bfloat16()
    eb = torch.randn(w, device=DEV) * 0.1
    x = torch.randn(rows, w, device=DEV).bfloat16()
    mean = torch.randn(w, device=DEV) * 0.1
    inv = torch.rand(w, device=DEV) + 0.5
    bw = torch.rand(w, device=DEV) + 0.5
    bb = torch.randn(w, device=DEV) * 0.1
    (o0, s0), (o1, s1) = both(C, lambda: C.gemm_xl_conv(dz, Bb, "bnbwd", bn_x=x, mean=mean, invstd=inv, weight=bw,
                                                        bias=bb, a2=a, ebias=eb))
    torch.testing.assert_close(o1.float(), o0.float(), atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(s1[:2 * w], s0[:2 * w], atol=2e-2 * rows ** 0.5, rtol=1e-3)
    # (no fp32 mask oracle here: an fma vs mul+add difference flips the ReLU
    # mask of the rare x * scale + shift within 1e-7 of zero)
    ref = torch.cat([dz, a], 1).float() @ Bb.float().t() + eb
    live = o1.float() != 0
    torch.testing.assert_close(o1.float()[live], ref[live], atol=6e-2, rtol=2e-2)


@pytest.mark.parametrize("mode", ["store", "bias"])
def test_gemm_xl_plain_tail(C, mode):
    torch.manual_seed(3)
    M, K, N = 257 * 256 - 11, 1024, 256
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    kw = {"bias": bias} if mode == "bias" else {}
    c0, c1 = both(C, lambda: C.gemm_xl(a, b, mode, **kw))
    torch.testing.assert_close(c1.float(), c0.float(), atol=3e-2, rtol=1e-2)
    ref = a.float() @ b.float().t() + (bias.float() if mode == "bias" else 0)
    torch.testing.assert_close(c1.float(), ref, atol=6e-2, rtol=2e-2)
