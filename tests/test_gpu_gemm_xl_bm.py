"""Trimmed tiles of the 256x256 ping-pong GEMM (csrc/gemm/gemm_xl.hip
pick_bm / set_gemm_xl_bm): an MFMA-bound grid whose last round of 256-row
tiles would be mostly empty runs 192..240-row tiles instead, so that the grid
fills whole rounds.  Each output element still accumulates the same K
sequence with the same MFMA, so every stored tensor must be BITWISE equal to
the 256-row launch; only the per-tile BN moment partials regroup (fp32 order).
Covered: every epilogue the ping-pong kernel runs (plain / bias / GELU /
GELU' + column sums / residual; conv moments / add / BN backward with x, with
y; the two-source folded dgrad; the stride-phase dgrad's row map), row counts
that leave a partial last tile, and the auto choice on the shapes it exists
for."""
import pytest
import torch

from distributed_model_parallel_amd import _native

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last
BMS = [240, 224, 208, 192]


@pytest.fixture
def C():
    c = _native.require("gemm_xl bm tests")
    # the 8-wave ping-pong kernel (PIPE 10) is the one with trimmed tiles; these
    # small grids would otherwise take 128-wide tiles (pick_bn)
    c.set_gemm_xl_bn(256, 10)
    yield c
    c.set_gemm_xl_bm(0)
    c.set_gemm_xl_bn(0)


def run(C, bm, fn):
    C.set_gemm_xl_bm(bm)
    out = fn()
    torch.cuda.synchronize()
    return out


def wmat(w):
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


def test_pick_bm_auto(C):
    C.set_gemm_xl_bm(0)
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("the expected choices assume 256 CUs")
    assert C.get_gemm_xl_bm(401408, 256, 2304) == 224   # layer-3 3x3 at batch 2048: 6.1 -> 7 full rounds
    assert C.get_gemm_xl_bm(100352, 512, 4608) == 208   # layer-4 3x3: 3.06 rounds
    assert C.get_gemm_xl_bm(50432, 768, 2304) == 208    # ViT qkv data gradient: 2.3 rounds
    assert C.get_gemm_xl_bm(50432, 2304, 768) == 256    # ViT qkv forward: 6.9 rounds already
    assert C.get_gemm_xl_bm(401408, 1024, 256) == 256   # short K: HBM-bound, never trimmed
    C.set_gemm_xl_bm(-1)
    assert C.get_gemm_xl_bm(401408, 256, 2304) == 256


@pytest.mark.parametrize("bm", BMS)
@pytest.mark.parametrize("mode", ["store", "bias", "bias_gelu", "bias_res"])
def test_gemm_xl_plain_bitwise(C, bm, mode):
    torch.manual_seed(0)
    M, K, N = 40 * 256 + 37, 768, 768
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    kw = {}
    if mode != "store":
        kw["bias"] = bias
    if mode == "bias_res":
        kw["residual"] = res
    aux0 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux1 = torch.empty_like(aux0)
    c0 = run(C, -1, lambda: C.gemm_xl(a, b, mode, aux=aux0 if mode == "bias_gelu" else None, **kw))
    c1 = run(C, bm, lambda: C.gemm_xl(a, b, mode, aux=aux1 if mode == "bias_gelu" else None, **kw))
    assert torch.equal(c0, c1)
    if mode == "bias_gelu":
        assert torch.equal(aux0, aux1)
    ref = a.float() @ b.float().t() + (bias.float() if mode != "store" else 0)
    if mode == "bias_res":
        ref = ref.bfloat16().float() + res.float()
    if mode != "bias_gelu":
        torch.testing.assert_close(c1.float(), ref, atol=6e-2, rtol=2e-2)


@pytest.mark.parametrize("bm", [224, 192])
def test_gemm_xl_dgelu_bgrad(C, bm):
    torch.manual_seed(1)
    M, K, N = 30 * 256 + 5, 1024, 512
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    aux = torch.randn(M, N, device=DEV).bfloat16()
    d0, g0 = run(C, -1, lambda: C.gemm_xl_dgelu_bgrad(a, b, aux))
    d1, g1 = run(C, bm, lambda: C.gemm_xl_dgelu_bgrad(a, b, aux))
    assert torch.equal(d0, d1)
    torch.testing.assert_close(g1, d1.float().sum(0), atol=2e-2 * M ** 0.5, rtol=1e-3)
    torch.testing.assert_close(g1, g0, atol=1e-2 * M ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("bm", [224, 208])
@pytest.mark.parametrize("n,c,h", [(41, 256, 14), (23, 512, 7)])
def test_conv_xl_moments_add_bnbwd(C, bm, n, c, h):
    torch.manual_seed(2)
    rows = n * h * h
    x = torch.randn(n, c, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = wmat((torch.randn(c, c, 3, 3, device=DEV) * 0.03).bfloat16())
    (y0, s0) = run(C, -1, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"))
    (y1, s1) = run(C, bm, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"))
    assert torch.equal(y0, y1)
    torch.testing.assert_close(s1[:2 * c], s0[:2 * c], atol=1e-2 * rows ** 0.5, rtol=1e-4)
    assert s1[2 * c].item() == rows
    f = y1.float()
    torch.testing.assert_close(s1[:c].float(), f.sum(0).double().float(), atol=2e-2 * rows ** 0.5, rtol=1e-3)
    res = torch.randn(rows, c, device=DEV).bfloat16()
    a0, _ = run(C, -1, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "add", residual=res))
    a1, _ = run(C, bm, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "add", residual=res))
    assert torch.equal(a0, a1)
    bx = torch.randn(rows, c, device=DEV).bfloat16()
    by = torch.relu(torch.randn(rows, c, device=DEV)).bfloat16()
    mean = torch.randn(c, device=DEV) * 0.1
    inv = torch.rand(c, device=DEV) + 0.5
    bw = torch.rand(c, device=DEV) + 0.5
    bb = torch.randn(c, device=DEV) * 0.1
    for kw in ({"bn_x": bx, "mean": mean, "invstd": inv, "weight": bw, "bias": bb},
               {"bn_x": bx, "bn_y": by, "mean": mean}, {"bn_y": by}):
        g0, t0 = run(C, -1, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "bnbwd", residual=res, **kw))
        g1, t1 = run(C, bm, lambda: C.conv_xl(x, w, 3, 3, 1, 1, h, h, "bnbwd", residual=res, **kw))
        assert torch.equal(g0, g1)
        torch.testing.assert_close(t1[:2 * c], t0[:2 * c], atol=1e-2 * rows ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("bm", [240, 192])
def test_gemm_xl_conv_fold_dgrad(C, bm):
    """The folded dgrad: two-source A ([dz | a]), ebias, BN backward, K = 1280."""
    torch.manual_seed(3)
    w, rows = 256, 37 * 256 - 9
    dz = torch.randn(rows, 4 * w, device=DEV).bfloat16()
    a = torch.randn(rows, w, device=DEV).bfloat16()
    Bb = (torch.randn(w, 5 * w, device=DEV) * 0.03).bfloat16()
    eb = torch.randn(w, device=DEV) * 0.1
    x = torch.randn(rows, w, device=DEV).bfloat16()
    mean = torch.randn(w, device=DEV) * 0.1
    inv = torch.rand(w, device=DEV) + 0.5
    bw = torch.rand(w, device=DEV) + 0.5
    bb = torch.randn(w, device=DEV) * 0.1
    f = lambda: C.gemm_xl_conv(dz, Bb, "bnbwd", bn_x=x, mean=mean, invstd=inv, weight=bw, bias=bb, a2=a, ebias=eb)
    o0, s0 = run(C, -1, f)
    o1, s1 = run(C, bm, f)
    assert torch.equal(o0, o1)
    torch.testing.assert_close(s1[:2 * w], s0[:2 * w], atol=1e-2 * rows ** 0.5, rtol=1e-4)


@pytest.mark.parametrize("bm", [224, 208])
def test_conv_xl_dgrad_s2_row_map(C, bm):
    """The stride-phase data gradient writes through an output row map."""
    from distributed_model_parallel_amd.ops import conv_igemm
    torch.manual_seed(4)
    n, cin, cout, hi = 19, 256, 512, 14
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.03).bfloat16()
    dy = torch.randn(n, cout, hi // 2, hi // 2, device=DEV).bfloat16().contiguous(memory_format=CL)
    wph = conv_igemm._phase_weights(w)
    d0 = run(C, -1, lambda: C.conv_xl_dgrad_s2(dy, wph, hi, hi))
    d1 = run(C, bm, lambda: C.conv_xl_dgrad_s2(dy, wph, hi, hi))
    assert torch.equal(d0, d1)


# ---- 4-wave kernel (PIPE 11, the default): 224-row tiles (7 MFMA blocks per
# wave, gemm_xl_w4_kernel<EPI, SRC, 7>) against its 256-row tiles, bitwise.

@pytest.fixture
def C4():
    c = _native.require("gemm_xl bm tests")
    c.set_gemm_xl_bn(256, 11)
    yield c
    c.set_gemm_xl_bm(0)
    c.set_gemm_xl_bn(0)


def test_pick_bm_w4_auto(C4):
    C4.set_gemm_xl_bm(0)
    if torch.cuda.get_device_properties(0).multi_processor_count != 256:
        pytest.skip("the expected choices assume 256 CUs")
    assert C4.get_gemm_xl_bm(50432, 768, 3072) == 224     # ViT N = 768: 591 tiles (3 rounds) -> 678 (3 rounds)
    assert C4.get_gemm_xl_bm(401408, 256, 2304) == 224    # ResNet-50 layer-3 3x3: 1568 -> 1792 tiles, 7 rounds
    assert C4.get_gemm_xl_bm(100352, 512, 4608) == 224    # layer-4 3x3: 784 -> 896 tiles, 4 rounds
    assert C4.get_gemm_xl_bm(50432, 2304, 768) == 256     # ViT qkv forward: 7 rounds either way
    C4.set_gemm_xl_bm(-1)
    assert C4.get_gemm_xl_bm(50432, 768, 3072) == 256


@pytest.mark.parametrize("mode", ["store", "bias", "bias_gelu", "bias_res"])
def test_w4_trimmed_plain_bitwise(C4, mode):
    torch.manual_seed(5)
    M, K, N = 40 * 224 + 37, 768, 768
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    bias = torch.randn(N, device=DEV).bfloat16()
    res = torch.randn(M, N, device=DEV).bfloat16()
    kw = {}
    if mode != "store":
        kw["bias"] = bias
    if mode == "bias_res":
        kw["residual"] = res
    aux0 = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    aux1 = torch.empty_like(aux0)
    c0 = run(C4, 256, lambda: C4.gemm_xl(a, b, mode, aux=aux0 if mode == "bias_gelu" else None, **kw))
    c1 = run(C4, 224, lambda: C4.gemm_xl(a, b, mode, aux=aux1 if mode == "bias_gelu" else None, **kw))
    assert torch.equal(c0, c1)
    if mode == "bias_gelu":
        assert torch.equal(aux0, aux1)
    ref = a.float() @ b.float().t() + (bias.float() if mode != "store" else 0)
    if mode == "bias_res":
        ref = ref.bfloat16().float() + res.float()
    if mode != "bias_gelu":
        torch.testing.assert_close(c1.float(), ref, atol=6e-2, rtol=2e-2)


def test_w4_trimmed_dgelu_bgrad(C4):
    torch.manual_seed(6)
    M, K, N = 30 * 224 + 5, 1024, 512
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    aux = torch.randn(M, N, device=DEV).bfloat16()
    d0, g0 = run(C4, 256, lambda: C4.gemm_xl_dgelu_bgrad(a, b, aux))
    d1, g1 = run(C4, 224, lambda: C4.gemm_xl_dgelu_bgrad(a, b, aux))
    assert torch.equal(d0, d1)
    torch.testing.assert_close(g1, d1.float().sum(0), atol=2e-2 * M ** 0.5, rtol=1e-3)


@pytest.mark.parametrize("n,c,h", [(41, 256, 14), (23, 512, 7)])
def test_w4_trimmed_conv_moments_store(C4, n, c, h):
    """3x3 tap gather (SRC 2) with the moments epilogue and the plain store,
    plus the stride-phase dgrad's output row map."""
    torch.manual_seed(7)
    rows = n * h * h
    x = torch.randn(n, c, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w = wmat((torch.randn(c, c, 3, 3, device=DEV) * 0.03).bfloat16())
    (y0, s0) = run(C4, 256, lambda: C4.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"))
    (y1, s1) = run(C4, 224, lambda: C4.conv_xl(x, w, 3, 3, 1, 1, h, h, "moments"))
    assert torch.equal(y0, y1)
    f = y1.float()
    torch.testing.assert_close(s1[:c].float(), f.sum(0), atol=2e-2 * rows ** 0.5, rtol=1e-3)
    torch.testing.assert_close(s1[c:2 * c].float(), (f * f).sum(0), atol=2e-2 * rows ** 0.5, rtol=1e-3)
    assert s1[2 * c].item() == rows
    ref = torch.nn.functional.conv2d(x.float(), (w.float().reshape(c, 3, 3, c).permute(0, 3, 1, 2)), padding=1)
    torch.testing.assert_close(y1.float(), ref.permute(0, 2, 3, 1).reshape(rows, c), atol=6e-2, rtol=2e-2)
    (z0, _) = run(C4, 256, lambda: C4.conv_xl(x, w, 3, 3, 1, 1, h, h, "store"))
    (z1, _) = run(C4, 224, lambda: C4.conv_xl(x, w, 3, 3, 1, 1, h, h, "store"))
    assert torch.equal(z0, z1) and torch.equal(z1, y1)
    from distributed_model_parallel_amd.ops import conv_igemm
    wc = (torch.randn(2 * c, c, 3, 3, device=DEV) * 0.03).bfloat16()
    dy = torch.randn(n, 2 * c, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    wph = conv_igemm._phase_weights(wc)
    d0 = run(C4, 256, lambda: C4.conv_xl_dgrad_s2(dy, wph, 2 * h, 2 * h))
    d1 = run(C4, 224, lambda: C4.conv_xl_dgrad_s2(dy, wph, 2 * h, 2 * h))
    assert torch.equal(d0, d1)


@pytest.mark.parametrize("n,cin,h,stride", [(37, 128, 56, 2), (9, 64, 28, 1), (5, 128, 28, 1)])
def test_w4_n128_conv_moments(n, cin, h, stride):
    """Cout = 128 convs on the 256 x 128 tile (WN = 1): output and fused moments
    against an fp32 conv of the same bf16 operands."""
    C = _native.require("gemm_xl n128")
    torch.manual_seed(8)
    cout = 128
    x = torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL)
    w4 = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.05).bfloat16()
    ho = (h + 2 - 3) // stride + 1
    rows = n * ho * ho
    y, s = C.conv_xl(x, wmat(w4), 3, 3, stride, 1, ho, ho, "moments")
    torch.cuda.synchronize()
    ref = torch.nn.functional.conv2d(x.float(), w4.float(), stride=stride, padding=1)
    ref2 = ref.permute(0, 2, 3, 1).reshape(rows, cout)
    torch.testing.assert_close(y.float(), ref2, atol=6e-2, rtol=2e-2)
    f = y.float()
    torch.testing.assert_close(s[:cout].float(), f.sum(0), atol=2e-2 * rows ** 0.5, rtol=1e-3)
    torch.testing.assert_close(s[cout:2 * cout].float(), (f * f).sum(0), atol=2e-2 * rows ** 0.5, rtol=1e-3)
    assert s[2 * cout].item() == rows
    z, _ = C.conv_xl(x, wmat(w4), 3, 3, stride, 1, ho, ho, "store")
    assert torch.equal(z, y)


def test_w4_n128_plain():
    C = _native.require("gemm_xl n128")
    torch.manual_seed(9)
    M, K, N = 13 * 256 + 77, 1152, 128
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.03).bfloat16()
    c = C.gemm_xl(a, b, "store")
    torch.testing.assert_close(c.float(), a.float() @ b.float().t(), atol=6e-2, rtol=2e-2)
