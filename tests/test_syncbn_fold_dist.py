"""SyncBatchNorm through the BN fold at world size 2 and 4 (gloo, CPU, fp64):
VERDICT r3 missing item 2.  The fold's distributed algebra -- forward moments
[W s, W G W^T, rows] all-reduced, backward [sum dz, sum dz (y - mean)]
all-reduced while dgamma / dbeta / dW / da stay local contributions -- must
make W ranks x b samples equal ONE process running plain training-mode BN on
the concatenated W*b batch: outputs, running statistics (every rank) and
every gradient (input gradients per slice, parameter gradients summed over
ranks, as DDP would).  Covers the bottleneck's bn2 (out_moments) -> conv3 +
bn3 fold with a residual, and the downsample variant (bn3 and bn_d folded into
one GEMM over [a | x_s], stride 2).  ``force=True`` runs the fold's CPU path,
the same algebra the GPU kernels implement (tests/test_gpu_bn_fold.py pins
kernels against it)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from tests.dist_utils import run_world

N_PER, C, CX, COUT, H = 2, 8, 16, 32, 4


def _globals(world, seed):
    g = torch.Generator().manual_seed(seed)
    d = dict(
        raw=torch.randn(world * N_PER, C, H, H, generator=g, dtype=torch.float64),
        x=torch.randn(world * N_PER, CX, 2 * H, 2 * H, generator=g, dtype=torch.float64),
        res=torch.randn(world * N_PER, COUT, H, H, generator=g, dtype=torch.float64),
        up=torch.randn(world * N_PER, COUT, H, H, generator=g, dtype=torch.float64),
        w3=torch.randn(COUT, C, 1, 1, generator=g, dtype=torch.float64) * 0.5,
        wd=torch.randn(COUT, CX, 1, 1, generator=g, dtype=torch.float64) * 0.4,
    )
    for name, n in (("bn2", C), ("bn3", COUT), ("bnd", COUT)):
        d[name + "_w"] = torch.rand(n, generator=g, dtype=torch.float64) + 0.5
        d[name + "_b"] = torch.randn(n, generator=g, dtype=torch.float64) * 0.3
    return d


def _sbn(n, act, w, b):
    from distributed_model_parallel_amd.parallel.sync_batchnorm import SyncBatchNorm
    m = SyncBatchNorm(n, act=act).double()
    with torch.no_grad():
        m.weight.copy_(w)
        m.bias.copy_(b)
    m.running_mean = m.running_mean.float()  # fp32 running stats, as the native BN keeps them
    m.running_var = m.running_var.float()
    return m


def _worker(rank, world, downsample):
    from distributed_model_parallel_amd.ops.bn_fold import conv1x1_bn_fold
    from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1
    d = _globals(world, 11)
    sl = slice(rank * N_PER, (rank + 1) * N_PER)
    cl = torch.channels_last
    bn2 = _sbn(C, "relu", d["bn2_w"], d["bn2_b"])
    bn3 = _sbn(COUT, "relu", d["bn3_w"], d["bn3_b"])
    conv3 = Conv1x1(C, COUT).double()
    with torch.no_grad():
        conv3.weight.copy_(d["w3"])
    raw = d["raw"][sl].contiguous(memory_format=cl).requires_grad_(True)
    a2, asums = bn2(raw, out_moments=True)
    if downsample:
        cd = Conv1x1(CX, COUT, 2).double()
        with torch.no_grad():
            cd.weight.copy_(d["wd"])
        bnd = _sbn(COUT, None, d["bnd_w"], d["bnd_b"])
        x = d["x"][sl].contiguous(memory_format=cl).requires_grad_(True)
        out = conv1x1_bn_fold(conv3, bn3, a2, asums, force=True, downsample=nn.Sequential(cd, bnd), x=x)
    else:
        res = d["res"][sl].contiguous(memory_format=cl).requires_grad_(True)
        out = conv1x1_bn_fold(conv3, bn3, a2, asums, res, force=True)
    (out * d["up"][sl]).sum().backward()
    r = dict(out=out.detach(), raw_g=raw.grad, w3_g=conv3.weight.grad,
             bn2=(bn2.weight.grad, bn2.bias.grad, bn2.running_mean.clone(), bn2.running_var.clone()),
             bn3=(bn3.weight.grad, bn3.bias.grad, bn3.running_mean.clone(), bn3.running_var.clone()))
    if downsample:
        r.update(x_g=x.grad, wd_g=cd.weight.grad,
                 bnd=(bnd.weight.grad, bnd.bias.grad, bnd.running_mean.clone(), bnd.running_var.clone()))
    else:
        r.update(res_g=res.grad)
    return r


def _reference(world, downsample):
    """One process, plain training-mode BN over the whole W*b batch."""
    d = _globals(world, 11)
    leaf = lambda t: t.clone().requires_grad_(True)  # noqa: E731
    raw, w3 = leaf(d["raw"]), leaf(d["w3"])
    p = {k: leaf(d[k]) for k in d if k.endswith("_w") or k.endswith("_b")}
    stats = {n: (torch.zeros(c, dtype=torch.float64), torch.ones(c, dtype=torch.float64))
             for n, c in (("bn2", C), ("bn3", COUT), ("bnd", COUT))}
    a2 = F.relu(F.batch_norm(raw, *stats["bn2"], p["bn2_w"], p["bn2_b"], True, 0.1, 1e-5))
    y = F.batch_norm(F.conv2d(a2, w3), *stats["bn3"], p["bn3_w"], p["bn3_b"], True, 0.1, 1e-5)
    out = dict()
    if downsample:
        x, wd = leaf(d["x"]), leaf(d["wd"])
        r = F.batch_norm(F.conv2d(x, wd, stride=2), *stats["bnd"], p["bnd_w"], p["bnd_b"], True, 0.1, 1e-5)
        o = F.relu(y + r)
    else:
        res = leaf(d["res"])
        o = F.relu(y + res)
    (o * d["up"]).sum().backward()
    out.update(out=o.detach(), raw_g=raw.grad, w3_g=w3.grad, stats=stats, p=p)
    if downsample:
        out.update(x_g=x.grad, wd_g=wd.grad)
    else:
        out.update(res_g=res.grad)
    return out


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("downsample", [False, True], ids=["residual", "downsample_s2"])
def test_syncbn_fold_equals_single_process_bn(world, downsample):
    res = run_world(_worker, world, downsample)
    ref = _reference(world, downsample)
    tol = dict(rtol=1e-5, atol=1e-6)
    cat = lambda k: torch.cat([r[k] for r in res])  # noqa: E731
    ssum = lambda f: sum(f(r) for r in res)  # noqa: E731
    torch.testing.assert_close(cat("out"), ref["out"], **tol)
    torch.testing.assert_close(cat("raw_g"), ref["raw_g"], **tol)
    torch.testing.assert_close(ssum(lambda r: r["w3_g"]), ref["w3_g"], **tol)
    names = ["bn2", "bn3"] + (["bnd"] if downsample else [])
    for n in names:
        torch.testing.assert_close(ssum(lambda r: r[n][0]), ref["p"][n + "_w"].grad, **tol, msg=f"{n} dgamma")
        torch.testing.assert_close(ssum(lambda r: r[n][1]), ref["p"][n + "_b"].grad, **tol, msg=f"{n} dbeta")
        for r in res:  # running statistics are the GLOBAL batch's, on every rank
            torch.testing.assert_close(r[n][2].double(), ref["stats"][n][0], rtol=1e-6, atol=1e-6)
            torch.testing.assert_close(r[n][3].double(), ref["stats"][n][1], rtol=1e-6, atol=1e-6)
    if downsample:
        torch.testing.assert_close(cat("x_g"), ref["x_g"], **tol)
        torch.testing.assert_close(ssum(lambda r: r["wd_g"]), ref["wd_g"], **tol)
    else:
        torch.testing.assert_close(cat("res_g"), ref["res_g"], **tol)
