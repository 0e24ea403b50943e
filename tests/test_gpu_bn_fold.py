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
    ref = (torch.cat([A, A2], 1).float() @ B.float().t()).bfloat16().float() + bias
    ref = ref.bfloat16().float() * (y.float() > 0)
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
    ref2 = (torch.cat([A, A2], 1).float() @ B.float().t()).bfloat16().float() + bias
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
    acc = (A.float() @ B.float().t()).bfloat16().float()
    ref = torch.relu(acc * sc + sh + R.float())
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


def _chain(bn2, conv3, bn3, nxt, raw, res, up):
    a2, asums = bn2(raw, out_moments=True)
    out = bn_fold.conv1x1_bn_fold(conv3, bn3, a2, asums, res)
    z = nxt(out)
    (z.float() * up).sum().backward()
    return out


@pytest.mark.parametrize("cin,hw,n", [(64, 56, 6), (128, 28, 16), (256, 14, 32), (512, 7, 64)])
def test_fold_chain_matches_fp32_reference(cin, hw, n):
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
    params32 = {k: v.detach().clone() for k, v in
                [("w2", bn2.weight), ("b2", bn2.bias), ("w3", conv3.weight), ("g3", bn3.weight),
                 ("be3", bn3.bias), ("wn", nxt.weight)]}
    for m in (conv3, nxt):
        m.weight.data = m.weight.data.bfloat16().contiguous(memory_format=torch.channels_last)
    raw = (torch.randn(n, cin, hw, hw, device=DEV) * 2 + 0.5).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    res = torch.randn(n, cout, hw, hw, device=DEV).bfloat16().contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    up = torch.randn(n, cin, hw, hw, device=DEV).contiguous(memory_format=torch.channels_last)
    before = bn_fold.stats()
    out = _chain(bn2, conv3, bn3, nxt, raw, res, up)
    after = bn_fold.stats()
    assert after["fold"] == before["fold"] + 1
    assert after["fold_fused_bwd"] == before["fold_fused_bwd"] + 1          # next conv masked dz
    assert after["fold_bnbwd_epilogue"] == before["fold_bnbwd_epilogue"] + 1  # bn2 reductions fused
    # fp32 stock reference from the same bf16 inputs / weights
    p = {k: v.float().requires_grad_(True) for k, v in params32.items()}
    p["w3"].data = conv3.weight.detach().float().contiguous()
    p["wn"].data = nxt.weight.detach().float().contiguous()
    r_raw = raw.detach().float().requires_grad_(True)
    r_res = res.detach().float().requires_grad_(True)
    a = F.relu(F.batch_norm(r_raw, None, None, p["w2"], p["b2"], True, 0.1, 1e-5))
    y = F.batch_norm(F.conv2d(a, p["w3"]), None, None, p["g3"], p["be3"], True, 0.1, 1e-5)
    o = F.relu(y + r_res)
    (F.conv2d(o, p["wn"]) * up).sum().backward()
    _check(out, o, 2e-2)
    _check(res.grad, r_res.grad, 5e-2)
    _check(raw.grad, r_raw.grad, 5e-2)
    _check(conv3.weight.grad, p["w3"].grad, 3e-2)
    _check(bn3.weight.grad, p["g3"].grad, 3e-2)
    _check(bn3.bias.grad, p["be3"].grad, 3e-2)
    _check(bn2.weight.grad, p["w2"].grad, 5e-2)
    _check(bn2.bias.grad, p["b2"].grad, 5e-2)
    # running statistics of bn3 from the Gram algebra vs the stock moments of y
    yd = F.conv2d(a.detach(), p["w3"].detach()).double()
    mean = yd.mean((0, 2, 3))
    var = yd.var((0, 2, 3), unbiased=True)
    torch.testing.assert_close(bn3.running_mean.double(), 0.1 * mean, rtol=2e-2, atol=2e-3)
    torch.testing.assert_close(bn3.running_var.double(), 0.9 + 0.1 * var, rtol=2e-2, atol=2e-3)


def test_bottleneck_fold_matches_unfused_model():
    """Two ResNet-50 layer-1 bottlenecks in bf16: fold on vs DMP's unfused
    native path (bn_fold.ENABLED off) -- outputs and every parameter gradient."""
    import copy
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(4)
    down = torch.nn.Sequential(Conv1x1(64, 256), BatchNormAct2d(256))
    net = cast_model(torch.nn.Sequential(Bottleneck(64, 64, 1, down), Bottleneck(256, 64))
                     .to(DEV).to(memory_format=torch.channels_last))
    ref = copy.deepcopy(net)
    net.train()
    ref.train()
    x = torch.randn(8, 64, 56, 56, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.randn(8, 256, 56, 56, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    before = bn_fold.stats()["fold"]
    x1 = x.clone().requires_grad_(True)
    y1 = net(x1)
    y1.backward(g)
    assert bn_fold.stats()["fold"] == before + 2
    old = bn_fold.ENABLED
    bn_fold.ENABLED = False
    try:
        x2 = x.clone().requires_grad_(True)
        y2 = ref(x2)
        y2.backward(g)
    finally:
        bn_fold.ENABLED = old
    assert bn_fold.stats()["fold"] == before + 2
    _check(y1, y2, 2e-2)
    _check(x1.grad, x2.grad, 5e-2)
    for (n1, p1), (_, p2) in zip(net.named_parameters(), ref.named_parameters()):
        _check(p1.grad, p2.grad, 6e-2, n1)
    for (n1, b1), (_, b2) in zip(net.named_buffers(), ref.named_buffers()):
        if b1.dtype.is_floating_point:
            _check(b1, b2, 2e-2, n1)


@pytest.mark.parametrize("cout,cin", [(256, 64), (512, 128), (1024, 256), (2048, 512)])
def test_fold_coefficient_kernels_match_fp64(cout, cin):
    """bn_fold_fwd / bn_fold_bwd_sums / bn_fold_bwd_coef against the same
    algebra in fp64 torch ops (the framework's CPU path)."""
    C = _native.require("fold kernels")
    torch.manual_seed(5)
    W = (torch.randn(cout, cin, device=DEV) * 0.05).bfloat16()
    a = torch.relu(torch.randn(4096, cin, device=DEV)).bfloat16()
    G = (a.double().t() @ a.double()).float()
    ad = a.double()
    asums = torch.cat([ad.sum(0), (ad * ad).sum(0), ad.new_tensor([4096.0])])
    sums, WG = C.bn_fold_fwd(W, G, asums)
    rs, rWG = bn_fold._fold_stats(W, G, asums[:cin], asums[2 * cin:])
    torch.testing.assert_close(WG.double(), rWG, rtol=1e-5, atol=1e-4)
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
    dW, dg, db, Bm, eb = C.bn_fold_bwd_coef(local, local, cnt, invstd, mean, gamma, D, WG, asums[:cin], W)
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
