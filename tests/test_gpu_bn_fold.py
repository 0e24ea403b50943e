"""BN fold on MI355X (ops/bn_fold.py) against fp32 PyTorch references.

1. the new kernel modes on their own: NT / xl GEMM with a second A source
   ([A | A2] along K), the affine+residual+ReLU epilogue of gemm_xl_conv,
   bnbwd with a per-column bias and without the BN input, and the BN apply
   pass's output moments;
2. the whole chain bn2(out_moments) -> fold(conv3, bn3, residual) -> next 1x1
   conv on every ResNet-50 bottleneck shape, so the fused paths all run
   (bn2's reductions in the folded dgrad epilogue, the next conv's epilogue
   masking dz for the fold) and are compared with the stock fp32 chain."""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops import bn_fold
from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def _check(a, b, tol, what=""):
    r = _rel(a, b)
    assert r < tol, f"{what}: relative error {r:.4f} >= {tol}"


@pytest.mark.parametrize("M,N,K1,K2,xl", [(3000, 64, 256, 64, False), (1000, 128, 512, 128, False),
                                         (777, 256, 1024, 256, False), (600, 512, 2048, 512, True),
                                         (700, 256, 256, 64, True)])
def test_two_source_gemm_bias_bnbwd(M, N, K1, K2, xl):
    C = _native.require("fold kernels")
    torch.manual_seed(0)
    A = torch.randn(M, K1, device=DEV).bfloat16()
    A2 = torch.randn(M, K2, device=DEV).bfloat16()
    B = (torch.randn(N, K1 + K2, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV)
    y = torch.relu(torch.randn(M, N, device=DEV)).bfloat16()          # mask source, no BN input
    ref = (torch.cat([A, A2], 1).float() @ B.float().t() + bias).bfloat16().float() * (y.float() > 0)
    if xl:
        dz, sums = C.gemm_xl_conv(A, B, "bnbwd", bn_y=y, a2=A2, ebias=bias)
    else:
        dz, sums = C.gemm_nt_bnbwd(A, B, None, None, y, None, None, None, None, a2=A2, ebias=bias)
    _check(dz, ref, 1e-2)
    torch.testing.assert_close(sums[:N], dz.double().sum(0), atol=1e-2, rtol=1e-4)
    assert float(sums[N:2 * N].abs().max()) == 0.0  # no BN input: only sum dz is reduced
    # plain two-source store through the affine epilogue (shift only)
    if xl:
        c2, _ = C.gemm_xl_conv(A, B, "affine", a2=A2, shift=bias)
    else:
        c2, _ = C.gemm_nt(A, B, mode="affine", epi_shift=bias, a2=A2)
    ref2 = torch.cat([A, A2], 1).float() @ B.float().t() + bias
    _check(c2, ref2, 1e-2)


@pytest.mark.parametrize("M,N,K", [(5000, 512, 128), (1200, 1024, 256), (300, 2048, 512)])
def test_xl_affine_residual_relu(M, N, K):
    C = _native.require("fold kernels")
    torch.manual_seed(1)
    A = torch.randn(M, K, device=DEV).bfloat16()
    B = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    R = torch.randn(M, N, device=DEV).bfloat16()
    sc = torch.rand(N, device=DEV) + 0.5
    sh = torch.randn(N, device=DEV)
    out, _ = C.gemm_xl_conv(A, B, "affine", residual=R, scale=sc, shift=sh, relu=True)
    acc = A.float() @ B.float().t()
    ref = torch.relu((acc * sc + sh).bfloat16().float() + R.float())  # affine on fp32 acc, then + R
    _check(out, ref, 1e-2)


def test_bn_apply_out_moments():
    C = _native.require("bn out moments")
    torch.manual_seed(2)
    for M, Cc in ((300_000, 64), (4097, 128), (100, 512)):
        x = torch.randn(M, Cc, device=DEV).bfloat16()
        xd = x.double()
        sums = torch.cat([xd.sum(0), (xd * xd).sum(0), xd.new_tensor([float(M)])])
        w = torch.rand(Cc, device=DEV) + 0.5
        b = torch.randn(Cc, device=DEV) * 0.3
        y, mean, inv, osums = C.bn_forward_apply(x, sums, w, b, None, None, 0.1, 1e-5, None, True, Cc,
                                                 None, True)
        yd = y.double()
        torch.testing.assert_close(osums[:Cc], yd.sum(0), rtol=1e-5, atol=1e-3)
        torch.testing.assert_close(osums[Cc:2 * Cc], (yd * yd).sum(0), rtol=1e-5, atol=1e-3)
        assert osums[2 * Cc].item() == M
        y0, _, _ = C.bn_forward_apply(x, sums, w, b, None, None, 0.1, 1e-5, None, True, Cc)
        assert torch.equal(y, y0)


def _chain(bn2, conv3, bn3, nxt, raw, res, up, fold=True):
    from distributed_model_parallel_amd.ops.fused import conv_bn
    if fold:
        a2, asums = bn2(raw, out_moments=True)
        out = bn_fold.conv1x1_bn_fold(conv3, bn3, a2, asums, res)
    else:
        out = conv_bn(conv3, bn3, bn2(raw), res)
    z = nxt(out)
    (z.float() * up).sum().backward()
    return out


@pytest.mark.parametrize("cin,hw,n", [(64, 56, 6), (128, 28, 16), (256, 14, 32), (512, 7, 64)])
def test_fold_chain_matches_fp32_reference(cin, hw, n):
    """Fold vs the unfused native bf16 chain, both measured against the fp32
    stock chain: the fold may not be less accurate than what it replaces."""
    import copy
    torch.manual_seed(3)
    cout = 4 * cin
    bn2 = BatchNormAct2d(cin, act="relu").to(DEV)
    conv3 = Conv1x1(cin, cout).to(DEV)
    bn3 = BatchNormAct2d(cout, act="relu").to(DEV)
    nxt = Conv1x1(cout, cin).to(DEV)
    with torch.no_grad():
        for bn in (bn2, bn3):
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.normal_(0, 0.2)
    for m in (conv3, nxt):
        m.weight.data = m.weight.data.bfloat16().contiguous(memory_format=torch.channels_last)
    mods_u = copy.deepcopy((bn2, conv3, bn3, nxt))
    raw0 = (torch.randn(n, cin, hw, hw, device=DEV) * 2 + 0.5).bfloat16().contiguous(memory_format=torch.channels_last)
    res0 = torch.randn(n, cout, hw, hw, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    up = torch.randn(n, cin, hw, hw, device=DEV).contiguous(memory_format=torch.channels_last)
    # fp32 stock reference from the same bf16 inputs / weights
    p = {"w2": bn2.weight, "b2": bn2.bias, "w3": conv3.weight, "g3": bn3.weight, "be3": bn3.bias, "wn": nxt.weight}
    p = {k: v.detach().float().clone().requires_grad_(True) for k, v in p.items()}
    r_raw = raw0.float().requires_grad_(True)
    r_res = res0.float().requires_grad_(True)
    a = F.relu(F.batch_norm(r_raw, None, None, p["w2"], p["b2"], True, 0.1, 1e-5))
    y = F.batch_norm(F.conv2d(a, p["w3"]), None, None, p["g3"], p["be3"], True, 0.1, 1e-5)
    o = F.relu(y + r_res)
    (F.conv2d(o, p["wn"]) * up).sum().backward()

    def run(mods, fold):
        raw = raw0.clone().requires_grad_(True)
        res = res0.clone().requires_grad_(True)
        out = _chain(*mods, raw, res, up, fold=fold)
        b2, c3, b3, _ = mods
        return {"out": (out, o), "res": (res.grad, r_res.grad), "raw": (raw.grad, r_raw.grad),
                "w3": (c3.weight.grad, p["w3"].grad), "g3": (b3.weight.grad, p["g3"].grad),
                "be3": (b3.bias.grad, p["be3"].grad), "w2": (b2.weight.grad, p["w2"].grad),
                "b2": (b2.bias.grad, p["b2"].grad)}, b3

    before = bn_fold.stats()
    got, bn3f = run((bn2, conv3, bn3, nxt), True)
    after = bn_fold.stats()
    assert after["fold"] == before["fold"] + 1
    assert after["fold_fused_bwd"] == before["fold_fused_bwd"] + 1          # next conv masked dz
    assert after["fold_bnbwd_epilogue"] == before["fold_bnbwd_epilogue"] + 1  # bn2 reductions fused
    ref, _ = run(mods_u, False)
    assert bn_fold.stats()["fold"] == after["fold"]
    errs = {k: (_rel(*got[k]), _rel(*ref[k])) for k in got}
    print(f"\n[fold vs unfused rel. error, cin={cin}] " + " ".join(f"{k}={a:.4f}/{b:.4f}" for k, (a, b) in errs.items()))
    for k, (e_fold, e_unf) in errs.items():
        # bn2's dgamma/dbeta are sums of O(M) noisy terms whose true value is small:
        # their relative errors are noise-dominated for both paths
        slack = 2.0 if k in ("w2", "b2") else 1.3
        assert e_fold < max(slack * e_unf, 1e-2), f"{k}: fold {e_fold:.4f} vs unfused {e_unf:.4f}"
    # running statistics of bn3 from the Gram algebra vs the stock moments of y
    yd = F.conv2d(a.detach(), p["w3"].detach()).double()
    mean = yd.mean((0, 2, 3))
    var = yd.var((0, 2, 3), unbiased=True)
    torch.testing.assert_close(bn3f.running_mean.double(), 0.1 * mean, rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(bn3f.running_var.double(), 0.9 + 0.1 * var, rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("low_rows", [False, True], ids=["default_routes", "strided_wgrad_xl"])
@pytest.mark.parametrize("cin,planes,stride,hw", [(64, 64, 1, 56), (256, 128, 2, 56), (512, 256, 2, 28),
                                                   (1024, 512, 2, 14), (1024, 512, 2, 4)])
def test_bottleneck_fold_matches_unfused_model(cin, planes, stride, hw, low_rows, monkeypatch):
    """A downsampling bottleneck + a plain one in bf16, fold on (bn3 folded; the
    first block's downsample conv + BN folded into the same GEMM) vs DMP's
    unfused native path (bn_fold.ENABLED off), each measured against the same
    blocks in fp32 stock PyTorch (reference_mode): the fold may not be less accurate."""
    import copy
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    from distributed_model_parallel_amd.ops import conv1x1 as c1
    from distributed_model_parallel_amd.utils.precision import cast_model
    if low_rows:  # these small batches through the batch-2048 routes (the 4-wave TN kernels)
        monkeypatch.setattr(c1, "_TN_XL_MIN_ROWS", 1024)
    torch.manual_seed(4)
    cout = planes * 4
    down = torch.nn.Sequential(Conv1x1(cin, cout, stride), BatchNormAct2d(cout))
    base = torch.nn.Sequential(Bottleneck(cin, planes, stride, down), Bottleneck(cout, planes)).to(DEV)
    net = cast_model(copy.deepcopy(base).to(memory_format=torch.channels_last))
    with torch.no_grad():
        for m in net.modules():
            if isinstance(m, BatchNormAct2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.normal_(0, 0.2)
    ref = copy.deepcopy(net)
    f32 = copy.deepcopy(net).float()
    for m in (net, ref, f32):
        m.train()
    nb = {56: 8, 28: 16, 14: 32, 4: 128}[hw]
    x = torch.relu(torch.randn(nb, cin, hw, hw, device=DEV)).bfloat16().contiguous(memory_format=torch.channels_last)
    ho = hw // stride
    g = torch.randn(nb, cout, ho, ho, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)

    def run(model, dtype):
        xi = x.to(dtype).clone().requires_grad_(True)
        y = model(xi)
        y.backward(g.to(dtype))
        return [y.float(), xi.grad.float()] + [p.grad.float() for p in model.parameters()]

    st0 = bn_fold.stats()
    got = run(net, torch.bfloat16)
    st1 = bn_fold.stats()
    assert st1["fold"] == st0["fold"] + 1 and st1["fold_ds"] == st0["fold_ds"] + 1
    if low_rows and stride != 1 and cin % 256 == 0 and nb * ho * ho >= 1024:  # strided branch: tap-gather TN
        assert st1.get("fold_ds_wgrad_xl", 0) == st0.get("fold_ds_wgrad_xl", 0) + 1
        assert st1.get("fold_ds_gram_xl", 0) == st0.get("fold_ds_gram_xl", 0) + 1
    if stride != 1:
        assert st1["fold_ds_compact"] == st0["fold_ds_compact"] + 1  # shortcut grad parked compact
    old = bn_fold.ENABLED
    bn_fold.ENABLED = False
    try:
        unf = run(ref, torch.bfloat16)
    finally:
        bn_fold.ENABLED = old
    with _native.reference_mode():
        gold = run(f32, torch.float32)
    names = ["out", "x.grad"] + [n for n, _ in net.named_parameters()]
    for n, a, b, r in zip(names, got, unf, gold):
        e_f, e_u = _rel(a, r), _rel(b, r)
        assert e_f < max(1.3 * e_u, 1e-2), f"{n}: fold {e_f:.4f} vs unfused {e_u:.4f} (fp32 reference)"
    for (n, b1), (_, b2) in zip(net.named_buffers(), ref.named_buffers()):
        if b1.dtype.is_floating_point:
            _check(b1, b2, 2e-2, n)


def test_fold_ds_kernels():
    """Strided colsum, Gram of a strided sample (gemm_tn a_mapped), the
    scale-concat operand and the two-source GEMMs with a mapped second source."""
    C = _native.require("fold kernels")
    torch.manual_seed(6)
    n, hi, cx, cin, cout, s = 4, 14, 256, 128, 512, 2
    ho = hi // s
    geom = [s, ho, ho, hi, hi]
    x = torch.relu(torch.randn(n, hi, hi, cx, device=DEV)).bfloat16()
    x2 = x.view(-1, cx)
    xs = x[:, ::s, ::s].reshape(-1, cx)
    for mp, rows in ((geom, xs), ([], x2)):
        m = C.bn_fold_colsum(x2, mp)
        rd = rows.double()
        torch.testing.assert_close(m[:cx], rd.sum(0), rtol=1e-5, atol=1e-2)
        torch.testing.assert_close(m[cx:2 * cx], (rd * rd).sum(0), rtol=1e-5, atol=1e-2)
        assert m[2 * cx].item() == rows.shape[0]
    G = C.gemm_tn(x2, x2, torch.float32, b_map=geom, a_mapped=True)
    _check(G, xs.double().t() @ xs.double(), 1e-5)
    W3 = (torch.randn(cout, cin, device=DEV) * 0.05).bfloat16()
    Wd = (torch.randn(cout, cx, device=DEV) * 0.05).bfloat16()
    s3, t3, sd, td = (torch.randn(cout, device=DEV) for _ in range(4))
    Bf, sh = C.bn_fold_scale_concat(W3, s3, t3, Wd, sd, td)
    torch.testing.assert_close(Bf.float(), torch.cat([s3[:, None] * W3.float(), sd[:, None] * Wd.float()], 1).bfloat16().float())
    torch.testing.assert_close(sh, t3 + td)
    a = torch.relu(torch.randn(n * ho * ho, cin, device=DEV)).bfloat16()
    ref = torch.relu(torch.cat([a, xs], 1).float() @ Bf.float().t() + sh)
    out_nt, _ = C.gemm_nt(a, Bf, mode="affine", epi_shift=sh, relu=True, a2=x2, a2_map=geom)
    out_xl, _ = C.gemm_xl_conv(a, Bf, "affine", shift=sh, relu=True, a2=x2, a2_map=geom)
    _check(out_nt, ref, 1e-2)
    _check(out_xl, ref, 1e-2)


@pytest.fixture(params=[2, 1, 0], ids=["tiled", "blas", "valu"])
def fold_mode(request):
    C = _native.require("fold kernels")
    old = C.get_fold_gemm()
    C.set_fold_gemm(request.param)
    yield request.param
    C.set_fold_gemm(old)


@pytest.mark.parametrize("cout,cin", [(256, 64), (512, 128), (1024, 256), (2048, 512), (2048, 1024), (512, 256)])
def test_fold_coefficient_kernels_match_fp64(cout, cin, fold_mode):
    """bn_fold_fwd / bn_fold_bwd_sums / bn_fold_bwd_coef against the same
    algebra in fp64 torch ops (the framework's CPU path), with the coefficient
    products on the tiled fp32 kernel, as library fp32 GEMMs and on the fused
    VALU kernels."""
    C = _native.require("fold kernels")
    torch.manual_seed(5)
    W = (torch.randn(cout, cin, device=DEV) * 0.05).bfloat16()
    a = torch.relu(torch.randn(4096, cin, device=DEV)).bfloat16()
    G = (a.double().t() @ a.double()).float()
    ad = a.double()
    asums = torch.cat([ad.sum(0), (ad * ad).sum(0), ad.new_tensor([4096.0])])
    sums, WG = C.bn_fold_fwd(W, G, asums)
    rs, rWG = bn_fold._fold_stats(W, G, asums[:cin], asums[2 * cin:])
    _check(WG, rWG, 1e-5)  # fp32 accumulation: relative to the matrix norm
    torch.testing.assert_close(sums, rs, rtol=1e-6, atol=1e-6)
    D = torch.randn(cout, cin, device=DEV)
    sdz = torch.randn(cout, device=DEV, dtype=torch.float64)
    mean = torch.randn(cout, device=DEV)
    invstd = torch.rand(cout, device=DEV) + 0.5
    gamma = torch.rand(cout, device=DEV) + 0.5
    local = C.bn_fold_bwd_sums(D, W, sdz, mean)
    Wd = W.double()
    sdzx = (D.double() * Wd).sum(1) - mean.double() * sdz
    torch.testing.assert_close(local, torch.cat([sdz, sdzx]), rtol=1e-9, atol=1e-9)
    cnt = asums[2 * cin:]
    dW, dg, db, Bm, eb = C.bn_fold_bwd_coef(local, local, cnt, invstd, mean, gamma, D, WG, asums, W)
    istd = invstd.double()
    al = istd * gamma.double()
    be = -al * istd * istd * sdzx / cnt
    cc = -al * sdz / cnt - be * mean.double()
    rdW = al[:, None] * D.double() + be[:, None] * WG.double() + cc[:, None] * asums[:cin][None, :]
    _check(dW, rdW, 1e-2)
    torch.testing.assert_close(dg.double(), sdzx * istd, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(db.double(), sdz, rtol=1e-5, atol=1e-5)
    _check(Bm[:, :cout], (al[:, None] * Wd).t(), 1e-2)
    _check(Bm[:, cout:], Wd.t() @ (be[:, None] * Wd), 1e-2)
    _check(eb, cc @ Wd, 1e-5)


@pytest.mark.parametrize("rows,c", [(100352, 2048), (1000, 256), (37, 64)])
def test_relu_mask_colsum_kernel(rows, c):
    """bn_fold_relu_mask: dz = [y > 0] dy and its fp64 column sums in one pass."""
    C = _native.require("test")
    torch.manual_seed(0)
    dy = torch.randn(rows, c, device="cuda").bfloat16()
    y = torch.relu(torch.randn(rows, c, device="cuda")).bfloat16()
    dz, s = C.bn_fold_relu_mask(dy, y)
    ref = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
    assert torch.equal(dz, ref)
    rd = ref.double()
    torch.testing.assert_close(s[:c], rd.sum(0), atol=1e-3 * rows ** 0.5, rtol=1e-5)
    torch.testing.assert_close(s[c:2 * c], (rd * rd).sum(0), atol=1e-3 * rows ** 0.5, rtol=1e-5)
    assert s[2 * c].item() == rows


@pytest.mark.parametrize("positive_w", [False, True], ids=["randn_w", "positive_w"])
def test_fold_statistics_at_headline_rows(positive_w):
    """the fold's BN3 statistics come from E[y^2] - E[y]^2
    over an fp32 Gram matrix accumulated across M = 2048 * 56 * 56 = 6.4 M rows
    (layer 1 of the batch-2048 bench).  Post-ReLU inputs (large mean / std)
    and -- the adversarial case -- all-positive weights give y a mean far
    above its spread, where the subtraction amplifies the Gram's fp32 error.
    The running statistics the fold writes must match an fp64 reference over
    the same bf16 operands."""
    torch.manual_seed(11)
    n, cin, cout, h = 2048, 64, 256, 56
    conv = Conv1x1(cin, cout).to(DEV).bfloat16()
    with torch.no_grad():
        w = torch.randn(cout, cin, 1, 1, device=DEV) * 0.2
        conv.weight.copy_(w.abs() if positive_w else w)
    conv = conv.to(memory_format=torch.channels_last)
    bn = BatchNormAct2d(cout, act="relu").to(DEV)  # fp32 running stats, bf16-free affine
    bn.weight.data = bn.weight.data.bfloat16()
    bn.bias.data = bn.bias.data.bfloat16()
    a = torch.relu(torch.randn(n, cin, h, h, device=DEV, dtype=torch.bfloat16) + 0.5)
    a = a.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    a2 = a.detach().permute(0, 2, 3, 1).reshape(-1, cin)
    # fp64 reference moments of the bf16 operands, chunked (6.4 M x 256 doubles would be 13 GB)
    W = conv.weight.detach().reshape(cout, cin).double()
    s1 = torch.zeros(cout, dtype=torch.float64, device=DEV)
    s2 = torch.zeros(cout, dtype=torch.float64, device=DEV)
    asum = torch.zeros(cin, dtype=torch.float64, device=DEV)
    asq = torch.zeros(cin, dtype=torch.float64, device=DEV)
    for r in range(0, a2.shape[0], 1 << 20):
        blk = a2[r:r + (1 << 20)].double()
        asum += blk.sum(0)
        asq += (blk * blk).sum(0)
        y = blk @ W.t()
        s1 += y.sum(0)
        s2 += (y * y).sum(0)
    m_rows = a2.shape[0]
    mean = s1 / m_rows
    var = s2 / m_rows - mean * mean
    a_sums = torch.cat([asum, asq, asum.new_tensor([float(m_rows)])])
    f0 = bn_fold.stats()["fold"]
    out = bn_fold.conv1x1_bn_fold(conv, bn, a, a_sums)
    assert bn_fold.stats()["fold"] == f0 + 1, "fold did not run"
    rm_ref = 0.1 * mean
    rv_ref = 0.9 + 0.1 * var * m_rows / (m_rows - 1)
    torch.testing.assert_close(bn.running_mean.double(), rm_ref, rtol=1e-4, atol=1e-5)
    rel_var = ((bn.running_var.double() - 0.9) / (rv_ref - 0.9) - 1).abs().max().item()
    ratio = (mean * mean / var).max().item()
    assert rel_var < 2e-3, f"variance relative error {rel_var:.2e} (max mean^2/var {ratio:.0f})"
    # and the normalised output of a sample of rows matches the fp64 statistics
    rows = torch.arange(0, m_rows, 9973, device=DEV)
    y = (a2[rows].double() @ W.t())
    ref = torch.relu((y - mean) / torch.sqrt(var + bn.eps) * bn.weight.double() + bn.bias.double())
    got = out.permute(0, 2, 3, 1).reshape(-1, cout)[rows].double()
    assert ((got - ref).norm() / ref.norm()).item() < 1e-2


@pytest.mark.parametrize("cout,cin", [(256, 64), (1024, 256), (2048, 512)])
def test_fold_fwd_finalize_matches_separate_launches(cout, cin):
    """bn_fold_fwd_finalize (moments + BN finalize in one launch) against
    bn_fold_fwd followed by bn_finalize: moments and step counter bitwise,
    coefficients and running statistics to fp32 rounding."""
    from distributed_model_parallel_amd import _native
    C = _native.require("bn_fold")
    torch.manual_seed(3)
    dev = "cuda"
    W = (torch.randn(cout, cin, device=dev) * 0.05).bfloat16()
    a = torch.relu(torch.randn(4096, cin, device=dev)).bfloat16()
    G = a.float().t() @ a.float()
    af = a.double()
    asums = torch.cat([af.sum(0), (af * af).sum(0), af.new_tensor([float(a.shape[0])])])
    w32 = torch.rand(cout, device=dev) + 0.5
    b32 = torch.randn(cout, device=dev) * 0.1
    outs = []
    for fused in (True, False):
        rm, rv = torch.zeros(cout, device=dev), torch.ones(cout, device=dev)
        nbt = torch.zeros(1, dtype=torch.long, device=dev)
        if fused:
            sums, WG, coef = C.bn_fold_fwd_finalize(W, G, asums, None, w32, b32, rm, rv, 0.1, 1e-5, nbt)
        else:
            sums, WG = C.bn_fold_fwd(W, G, asums)
            coef = C.bn_finalize(sums, w32, b32, rm, rv, 0.1, 1e-5, cout, nbt)
        torch.cuda.synchronize()
        outs.append((sums, WG, coef, rm, rv, nbt))
    (s1, w1, c1, rm1, rv1, n1), (s0, w0, c0, rm0, rv0, n0) = outs
    assert torch.equal(s1, s0) and torch.equal(w1, w0) and torch.equal(n1, n0)
    # (same formulas; only the compiler's fma contraction may differ between the two kernels)
    for x, y in ((c1, c0), (rm1, rm0), (rv1, rv0)):
        torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-7)
