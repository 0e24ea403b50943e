"""CPU oracle for the BN fold (ops/bn_fold.py): relu(bn(conv1x1(a)) + residual)
computed from the Gram matrix a^T a, colsum(a) and dz^T a must match the
stock composition F.conv2d -> F.batch_norm (training) -> add -> relu in
forward output, running statistics and every gradient (fp64, so the
algebra -- not rounding -- is what is tested)."""
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
from distributed_model_parallel_amd.ops.bn_fold import conv1x1_bn_fold
from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1


def _setup(seed, n=3, cin=8, cout=32, h=5, w=4, residual=True):
    g = torch.Generator().manual_seed(seed)
    conv = Conv1x1(cin, cout).double()
    bn = BatchNormAct2d(cout, act="relu").double()
    with torch.no_grad():
        conv.weight.copy_(torch.randn(cout, cin, 1, 1, generator=g, dtype=torch.float64) * 0.5)
        bn.weight.copy_(torch.rand(cout, generator=g, dtype=torch.float64) + 0.5)
        bn.bias.copy_(torch.randn(cout, generator=g, dtype=torch.float64) * 0.3)
        bn.running_mean.copy_(torch.randn(cout, generator=g, dtype=torch.float64))
    bn.running_mean = bn.running_mean.float()  # the fold (like the native BN) keeps fp32 running stats
    bn.running_var = bn.running_var.float()
    x = torch.randn(n, cin, h, w, generator=g, dtype=torch.float64)
    a = F.relu(x + 0.3).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    res = (torch.randn(n, cout, h, w, generator=g, dtype=torch.float64)
           .contiguous(memory_format=torch.channels_last).requires_grad_(True)) if residual else None
    up = torch.randn(n, cout, h, w, generator=g, dtype=torch.float64)
    return conv, bn, a, res, up


def _reference(conv, bn, a, res, up):
    rm, rv = bn.running_mean.double().clone(), bn.running_var.double().clone()
    wt = conv.weight.detach().clone().requires_grad_(True)
    gw = bn.weight.detach().clone().requires_grad_(True)
    gb = bn.bias.detach().clone().requires_grad_(True)
    a_ = a.detach().clone().requires_grad_(True)
    r_ = res.detach().clone().requires_grad_(True) if res is not None else None
    y = F.batch_norm(F.conv2d(a_, wt), rm, rv, gw, gb, True, bn.momentum, bn.eps)
    out = F.relu(y + r_ if r_ is not None else y)
    (out * up).sum().backward()
    return out.detach(), rm, rv, a_.grad, wt.grad, gw.grad, gb.grad, (r_.grad if r_ is not None else None)


def _colsum_moments(a):
    a2 = a.detach().permute(0, 2, 3, 1).reshape(-1, a.shape[1])
    return torch.cat([a2.sum(0), (a2 * a2).sum(0), a2.new_tensor([float(a2.shape[0])])])


def test_fold_matches_stock_composition():
    for seed, residual in ((0, True), (1, False), (2, True)):
        conv, bn, a, res, up = _setup(seed, residual=residual)
        ref = _reference(conv, bn, a, res, up)
        out = conv1x1_bn_fold(conv, bn, a, _colsum_moments(a), res, force=True)
        (out * up).sum().backward()
        torch.testing.assert_close(out, ref[0], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(bn.running_mean.double(), ref[1], rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(bn.running_var.double(), ref[2], rtol=1e-6, atol=1e-6)
        assert int(bn.num_batches_tracked) == 1
        torch.testing.assert_close(a.grad, ref[3], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(conv.weight.grad, ref[4], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(bn.weight.grad, ref[5], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(bn.bias.grad, ref[6], rtol=1e-5, atol=1e-6)
        if residual:
            torch.testing.assert_close(res.grad, ref[7], rtol=1e-5, atol=1e-6)


def test_fold_after_bn_out_moments_chain():
    """bn2 (out_moments) -> fold: the colsum comes from bn2's apply and the
    gradient flows back through bn2 exactly as in the stock chain."""
    g = torch.Generator().manual_seed(7)
    n, c, cout, h, w = 2, 8, 32, 4, 4
    bn2 = BatchNormAct2d(c, act="relu").double()
    conv, bn3, _, res, up = _setup(3, n=n, cin=c, cout=cout, h=h, w=w)
    with torch.no_grad():
        bn2.weight.copy_(torch.rand(c, generator=g, dtype=torch.float64) + 0.5)
        bn2.bias.copy_(torch.randn(c, generator=g, dtype=torch.float64) * 0.2)
    raw = torch.randn(n, c, h, w, generator=g, dtype=torch.float64).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    a2, asums = bn2(raw, out_moments=True)
    torch.testing.assert_close(asums, _colsum_moments(a2))
    out = conv1x1_bn_fold(conv, bn3, a2, asums, res, force=True)
    (out * up).sum().backward()
    # stock chain on clones
    raw_ = raw.detach().clone().requires_grad_(True)
    a_ = F.relu(F.batch_norm(raw_, None, None, bn2.weight.detach(), bn2.bias.detach(), True, 0.1, bn2.eps))
    ref = _reference(conv, bn3, a_, res, up)
    torch.testing.assert_close(out, ref[0], rtol=1e-5, atol=1e-6)
    a_2 = a_.detach().clone().requires_grad_(True)
    w_ = conv.weight.detach()
    y = F.batch_norm(F.conv2d(a_2, w_), None, None, bn3.weight.detach(), bn3.bias.detach(), True, 0.1, bn3.eps)
    o = F.relu(y + res.detach())
    (o * up).sum().backward()
    a_.backward(a_2.grad)
    torch.testing.assert_close(raw.grad, raw_.grad, rtol=1e-5, atol=1e-6)


def test_downsample_fold_matches_stock_composition():
    """bn3 and the downsample BN folded into one GEMM over [a | x_s]:
    relu(bn3(conv3(a)) + bn_d(conv_d(x, stride s))) against F.conv2d /
    F.batch_norm for stride 1 and 2 (fp64, CPU path of the same algebra)."""
    import torch.nn as nn
    for seed, stride in ((0, 1), (1, 2)):
        g = torch.Generator().manual_seed(seed)
        n, cin, cx, cout, hi = 2, 8, 16, 32, 6
        ho = (hi - 1) // stride + 1
        conv3, bn3, a, _, up = _setup(seed, n=n, cin=cin, cout=cout, h=ho, w=ho, residual=False)
        cd = Conv1x1(cx, cout, stride).double()
        bd = BatchNormAct2d(cout, act=None).double()
        with torch.no_grad():
            cd.weight.copy_(torch.randn(cout, cx, 1, 1, generator=g, dtype=torch.float64) * 0.4)
            bd.weight.copy_(torch.rand(cout, generator=g, dtype=torch.float64) + 0.5)
            bd.bias.copy_(torch.randn(cout, generator=g, dtype=torch.float64) * 0.3)
        bd.running_mean = bd.running_mean.float()
        bd.running_var = bd.running_var.float()
        ds = nn.Sequential(cd, bd)
        x = torch.randn(n, cx, hi, hi, generator=g, dtype=torch.float64).contiguous(
            memory_format=torch.channels_last).requires_grad_(True)
        # stock composition on clones
        a_ = a.detach().clone().requires_grad_(True)
        x_ = x.detach().clone().requires_grad_(True)
        w3 = conv3.weight.detach().clone().requires_grad_(True)
        wd = cd.weight.detach().clone().requires_grad_(True)
        p = [t.detach().clone().requires_grad_(True) for t in (bn3.weight, bn3.bias, bd.weight, bd.bias)]
        rm3, rv3 = bn3.running_mean.double().clone(), bn3.running_var.double().clone()
        rmd, rvd = bd.running_mean.double().clone(), bd.running_var.double().clone()
        y = F.batch_norm(F.conv2d(a_, w3), rm3, rv3, p[0], p[1], True, 0.1, 1e-5)
        r = F.batch_norm(F.conv2d(x_, wd, stride=stride), rmd, rvd, p[2], p[3], True, 0.1, 1e-5)
        o = F.relu(y + r)
        (o * up).sum().backward()
        out = conv1x1_bn_fold(conv3, bn3, a, _colsum_moments(a), force=True, downsample=ds, x=x)
        (out * up).sum().backward()
        tol = dict(rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(out, o, **tol)
        torch.testing.assert_close(a.grad, a_.grad, **tol)
        torch.testing.assert_close(x.grad, x_.grad, **tol)
        torch.testing.assert_close(conv3.weight.grad, w3.grad, **tol)
        torch.testing.assert_close(cd.weight.grad, wd.grad, **tol)
        for mine, ref in zip((bn3.weight, bn3.bias, bd.weight, bd.bias), p):
            torch.testing.assert_close(mine.grad, ref.grad, **tol)
        torch.testing.assert_close(bd.running_mean.double(), rmd, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(bd.running_var.double(), rvd, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(bn3.running_var.double(), rv3, rtol=1e-6, atol=1e-6)
