"""BN backward reductions fused into the consuming 1x1 conv's data-gradient
GEMM (EPI_BNBWD, ops/batchnorm.py BnBwdSlot) against fp32/fp64 PyTorch
references: the kernel on its own (mask from y or from the BN affine, with and
without the shortcut-gradient add), then whole blocks fused vs unfused."""
import copy

import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.ops import batchnorm as bnops
from distributed_model_parallel_amd.ops import bn_fold
from distributed_model_parallel_amd.ops import conv1x1
from distributed_model_parallel_amd.utils.precision import cast_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("M,N,K", [(4097, 64, 256), (1000, 256, 64), (333, 128, 512)])
@pytest.mark.parametrize("mask_from_y", [False, True])
@pytest.mark.parametrize("with_res", [False, True])
def test_gemm_nt_bnbwd_kernel(M, N, K, mask_from_y, with_res):
    C = _native.require("bnbwd test")
    torch.manual_seed(0)
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()      # W^T as the NT "B" operand
    x = torch.randn(M, N, device=DEV).bfloat16()               # BN input
    mean = x.float().mean(0)
    inv = torch.rand(N, device=DEV) + 0.5                       # BN invstd
    bw = torch.rand(N, device=DEV) + 0.5                        # BN weight, bias
    bb = torch.randn(N, device=DEV) * 0.5
    sc = inv * bw
    sh = bb - mean * sc
    res = torch.randn(M, N, device=DEV).bfloat16() if with_res else None
    y = torch.relu(x.float() * sc + sh + (res.float() if with_res else 0)).bfloat16() if mask_from_y else None
    dz, sums = C.gemm_nt_bnbwd(dy, wt, res, x, y, mean, None if mask_from_y else inv,
                               None if mask_from_y else bw, None if mask_from_y else bb)
    g = dy.float() @ wt.float().t()
    if with_res:
        g = g.bfloat16().float() + res.float()
    g = g.bfloat16().float()
    mask = (y.float() > 0) if mask_from_y else (x.float() * sc + sh > 0)
    ref = g * mask
    torch.testing.assert_close(dz.float(), ref, atol=0.05 * K ** 0.5 * 0.1 + 0.02, rtol=2e-2)
    # reductions are of the STORED dz (what the BN apply pass consumes)
    dzd = dz.double()
    torch.testing.assert_close(sums[:N], dzd.sum(0), atol=1e-2, rtol=1e-4)
    torch.testing.assert_close(sums[N:2 * N], (dzd * (x.double() - mean.double())).sum(0), atol=1e-2, rtol=1e-4)
    assert sums[2 * N].item() == M


def _run(blk, x, g):
    xi = x.detach().requires_grad_()
    y = blk(xi)
    y.backward(g)
    return y.float(), xi.grad.float(), {n: p.grad.float().clone() for n, p in blk.named_parameters()}


@pytest.mark.parametrize("stride", [1, 2])
def test_bottleneck_fused_bn_backward_matches_unfused(stride):
    """bn2 (mask from its affine, consumer conv3) and the previous block's bn3
    (mask from y, residual, consumer conv1 with the shortcut gradient) fused vs
    DMP_FUSE_BN_BWD off: same input / parameter gradients."""
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    cin, planes = 256, 64
    down = None
    if stride != 1:
        down = torch.nn.Sequential(conv1x1.Conv1x1(cin, planes * 4, stride), BatchNormAct2d(planes * 4))
    b1 = Bottleneck(cin, planes, 1)              # its bn3 output feeds b2's conv1
    b2 = Bottleneck(cin, planes, stride, down)
    net = cast_model(torch.nn.Sequential(b1, b2).to(DEV).to(memory_format=torch.channels_last))
    with torch.no_grad():
        for b in (b1, b2):
            b.bn3.weight.normal_(1.0, 0.1)
    ref = copy.deepcopy(net)
    net.train()
    ref.train()
    x = torch.randn(8, cin, 16, 16, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    gg = torch.randn(8, planes * 4, 16 // stride, 16 // stride, device=DEV).bfloat16() \
        .contiguous(memory_format=torch.channels_last)
    old = bnops._FUSE_BWD
    try:
        bnops._FUSE_BWD = False
        net2 = copy.deepcopy(ref)
        ya2, ga2, pa2 = _run(net2, x, gg)
        bnops._FUSE_BWD = True
        net3 = copy.deepcopy(ref)
        n0 = bnops._STATS["fused_bwd_moments"] + bn_fold.stats()["fold_fused_bwd"]
        c0 = conv1x1._STATS["compact_residual"]
        ya3, ga3, pa3 = _run(net3, x, gg)
        # b1.bn3 is folded through conv3 (ops/bn_fold.py): its fused backward counts there
        fused = bnops._STATS["fused_bwd_moments"] + bn_fold.stats()["fold_fused_bwd"] - n0
        compact = conv1x1._STATS["compact_residual"] - c0
    finally:
        bnops._FUSE_BWD = old
    assert fused >= 3, f"expected bn2 of both blocks and b1.bn3 fused, got {fused}"
    if stride != 1:  # the strided shortcut's dgrad reached b2.conv1's epilogue compact
        assert compact == 1, compact
    torch.testing.assert_close(ya3, ya2)
    cos = F.cosine_similarity(ga3.flatten(), ga2.flatten(), dim=0).item()
    assert cos > 0.995, cos
    for n in pa2:
        c = F.cosine_similarity(pa3[n].flatten(), pa2[n].flatten(), dim=0).item()
        assert c > 0.99, (n, c)


@pytest.mark.parametrize("xl", [False, True])
def test_bnbwd_compact_strided_residual(xl):
    """A stride-2 compact residual (res_map) == the same residual zero-expanded
    to full resolution, for both kernels."""
    C = _native.require("bnbwd test")
    torch.manual_seed(3)
    n, h, w, s, N, K = 3, 10, 9, 2, 256, 128
    ho, wo = (h + 1) // 2, (w + 1) // 2
    M = n * h * w
    dy = torch.randn(M, K, device=DEV).bfloat16()
    wt = (torch.randn(N, K, device=DEV) * 0.1).bfloat16()
    x = torch.randn(M, N, device=DEV).bfloat16()
    mean = x.float().mean(0)
    inv = torch.rand(N, device=DEV) + 0.5
    bb = torch.randn(N, device=DEV) * 0.5
    comp = torch.randn(n * ho * wo, N, device=DEV).bfloat16()
    full = torch.zeros(n, h, w, N, device=DEV).bfloat16()
    full[:, ::s, ::s] = comp.view(n, ho, wo, N)
    full = full.view(M, N)
    rmap = [s, ho, wo, h, w]
    if xl:
        a = C.gemm_xl_conv(dy, wt, "bnbwd", residual=comp, bn_x=x, mean=mean, invstd=inv, bias=bb, res_map=rmap)
        b = C.gemm_xl_conv(dy, wt, "bnbwd", residual=full, bn_x=x, mean=mean, invstd=inv, bias=bb)
    else:
        a = C.gemm_nt_bnbwd(dy, wt, comp, x, None, mean, inv, None, bb, rmap)
        b = C.gemm_nt_bnbwd(dy, wt, full, x, None, mean, inv, None, bb)
    torch.testing.assert_close(a[0], b[0])
    torch.testing.assert_close(a[1], b[1], atol=1e-6, rtol=1e-9)


def test_bottleneck_3x3_on_conv_xl_with_fused_bn1_backward():
    """Layer-3-width block: conv2 (3x3, 256 -> 256) forward and data gradient on
    conv_xl, its dgrad epilogue doing bn1's backward reductions -- vs conv_nt /
    MIOpen with the unfused BN backward."""
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    from distributed_model_parallel_amd.ops import conv_igemm
    torch.manual_seed(4)
    blk = Bottleneck(1024, 256, 1)
    net = cast_model(blk.to(DEV).to(memory_format=torch.channels_last))
    with torch.no_grad():
        net.bn1.weight.normal_(1.0, 0.1)
        net.bn1.bias.normal_(0.0, 0.1)
    net.train()
    x = torch.randn(4, 1024, 8, 8, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    gg = torch.randn(4, 1024, 8, 8, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    old = (bnops._FUSE_BWD, conv_igemm._XL3)
    try:
        bnops._FUSE_BWD, conv_igemm._XL3 = False, False
        ya, ga, pa = _run(copy.deepcopy(net), x, gg)
        bnops._FUSE_BWD, conv_igemm._XL3 = True, True
        s0 = dict(conv_igemm._STATS)
        n0 = bnops._STATS["fused_bwd_moments"]
        yb, gb, pb = _run(copy.deepcopy(net), x, gg)
        fused = bnops._STATS["fused_bwd_moments"] - n0
    finally:
        bnops._FUSE_BWD, conv_igemm._XL3 = old
    assert conv_igemm._STATS["xl_fwd"] > s0["xl_fwd"] and conv_igemm._STATS["xl_dgrad"] > s0["xl_dgrad"]
    assert conv_igemm._STATS["xl_bnbwd"] == s0["xl_bnbwd"] + 1
    assert fused >= 2, fused  # bn1 (via conv2 = conv_xl) and bn2 (via conv3)
    torch.testing.assert_close(yb, ya, atol=0.1, rtol=5e-2)
    cos = F.cosine_similarity(gb.flatten(), ga.flatten(), dim=0).item()
    assert cos > 0.995, cos
    for n in pa:
        c = F.cosine_similarity(pb[n].flatten(), pa[n].flatten(), dim=0).item()
        assert c > 0.99, (n, c)
