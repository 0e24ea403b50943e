"""BatchNormAct2d (CPU path) and SyncBatchNorm oracle over gloo.

SyncBN oracle: W ranks x b samples must match plain BN on the
W*b concatenated batch -- forward output, running statistics and input grads;
weight/bias grads averaged over ranks (what DDP does) equal the full-batch
grads divided by W for a mean loss... we compare sum-loss grads directly.
"""
import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d, batch_norm_act, reference_bn_act
from tests.dist_utils import run_world


@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("shape", [(4, 6, 5, 5), (16, 12)])
def test_bn_act_cpu_matches_reference(relu, res, shape):
    torch.manual_seed(0)
    C = shape[1]
    x = torch.randn(shape, dtype=torch.float64) * 3 + 1
    r = torch.randn(shape, dtype=torch.float64) if res else None
    w = torch.rand(C, dtype=torch.float64) + 0.5
    b = torch.randn(C, dtype=torch.float64)
    rm, rv = torch.zeros(C, dtype=torch.float64), torch.ones(C, dtype=torch.float64)
    rm2, rv2 = rm.clone(), rv.clone()
    args = [t.clone().requires_grad_() for t in (x, w, b)]
    ref = [t.clone().requires_grad_() for t in (x, w, b)]
    rr1 = r.clone().requires_grad_() if res else None
    rr2 = r.clone().requires_grad_() if res else None
    y = batch_norm_act(args[0], rm, rv, args[1], args[2], True, 0.1, 1e-5, relu=relu, residual=rr1)
    yr = reference_bn_act(ref[0], rm2, rv2, ref[1], ref[2], True, 0.1, 1e-5, relu=relu, residual=rr2)
    torch.testing.assert_close(y, yr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(rm, rm2)
    torch.testing.assert_close(rv, rv2)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    for a, bb in zip(args, ref):
        torch.testing.assert_close(a.grad, bb.grad.to(a.grad.dtype), atol=1e-5, rtol=1e-5)
    if res:
        torch.testing.assert_close(rr1.grad, rr2.grad)


def test_bn_module_eval_and_state_dict_compat():
    m = BatchNormAct2d(8, act="relu")
    ref = torch.nn.BatchNorm2d(8)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(2, 8, 3, 3)
    m.train(), ref.train()
    torch.testing.assert_close(m(x), F.relu(ref(x)))
    m.eval(), ref.eval()
    torch.testing.assert_close(m(x), F.relu(ref(x)))
    assert set(m.state_dict()) == set(ref.state_dict())


WORLD = 2


def _syncbn_worker(rank, world, relu):
    from distributed_model_parallel_amd.parallel.sync_batchnorm import SyncBatchNorm
    torch.manual_seed(0)
    full = torch.randn(world * 3, 4, 5, 5, dtype=torch.float64) * 2 + 0.3
    g = torch.randn(world * 3, 4, 5, 5, dtype=torch.float64)
    bn = SyncBatchNorm(4, act="relu" if relu else None).double()
    x = full[rank * 3:(rank + 1) * 3].clone().requires_grad_()
    y = bn(x)
    (y * g[rank * 3:(rank + 1) * 3]).sum().backward()
    return {"y": y.detach(), "dx": x.grad, "dw": bn.weight.grad, "db": bn.bias.grad,
            "rm": bn.running_mean.clone(), "rv": bn.running_var.clone()}


@pytest.mark.parametrize("relu", [False, True])
def test_syncbn_matches_full_batch_bn(relu):
    res = run_world(_syncbn_worker, WORLD, relu)
    torch.manual_seed(0)
    full = torch.randn(WORLD * 3, 4, 5, 5, dtype=torch.float64) * 2 + 0.3
    g = torch.randn(WORLD * 3, 4, 5, 5, dtype=torch.float64)
    ref = torch.nn.BatchNorm2d(4).double()
    x = full.clone().requires_grad_()
    y = ref(x)
    if relu:
        y = F.relu(y)
    (y * g).sum().backward()
    y_all = torch.cat([r["y"] for r in res])
    dx_all = torch.cat([r["dx"] for r in res])
    torch.testing.assert_close(y_all, y.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(dx_all, x.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(res[0]["rm"], ref.running_mean)
    torch.testing.assert_close(res[0]["rv"], ref.running_var)
    # per-rank weight/bias grads are local; their sum is the full-batch grad
    torch.testing.assert_close(res[0]["dw"] + res[1]["dw"], ref.weight.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(res[0]["db"] + res[1]["db"], ref.bias.grad, atol=1e-5, rtol=1e-5)


def test_convert_sync_batchnorm_keeps_params():
    from distributed_model_parallel_amd.models import resnet18
    from distributed_model_parallel_amd.parallel.sync_batchnorm import SyncBatchNorm
    m = resnet18(num_classes=10)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    m2 = SyncBatchNorm.convert_sync_batchnorm(m)
    assert sum(isinstance(x, SyncBatchNorm) for x in m2.modules()) == 20
    after = m2.state_dict()
    assert set(before) == set(after)
    for k in before:
        torch.testing.assert_close(before[k], after[k])
    assert m2.layer1[0].bn1.act == "relu"
