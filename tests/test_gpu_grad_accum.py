"""Micro-batch gradient accumulation inside the weight-gradient kernels
(ops/grad_accum.py): under ``accumulate_param_grads`` the
native ops add their parameter gradient into ``p.grad`` in the pass that
writes it (split-K reduce, depthwise column reduce, BN backward apply) and
return None to autograd.  Oracle: the same ops with autograd's
AccumulateGrad adds, and the fp32 PyTorch reference of the op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _twice(fn, params, accumulate):
    from distributed_model_parallel_amd.ops import grad_accum
    for p in params:
        p.grad = torch.zeros_like(p)
    before = grad_accum.stats()["kernel"]
    with grad_accum.accumulate_param_grads(accumulate):
        for i in range(2):
            fn(i)
    return [p.grad.clone() for p in params], grad_accum.stats()["kernel"] - before


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("n,cin,cout,h,stride", [(8, 64, 128, 16, 1), (64, 64, 64, 16, 1), (8, 96, 24, 16, 2)])
def test_conv1x1_wgrad_accumulates_in_kernel(n, cin, cout, h, stride):
    from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1
    torch.manual_seed(0)
    conv = Conv1x1(cin, cout, stride=stride).to(DEV, torch.bfloat16).to(memory_format=CL)
    xs = [torch.randn(n, cin, h, h, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    gs = [torch.randn(n, cout, (h - 1) // stride + 1, (h - 1) // stride + 1, device=DEV).bfloat16() for _ in range(2)]

    def fn(i):
        conv(xs[i]).backward(gs[i])
    (acc,), used = _twice(fn, [conv.weight], True)
    (ref,), used_ref = _twice(fn, [conv.weight], False)
    assert used == 2 and used_ref == 0
    w32 = conv.weight.detach().float().requires_grad_()
    for i in range(2):
        F.conv2d(xs[i].float(), w32, None, stride).backward(gs[i].float())
    assert _rel(acc, w32.grad) < 1e-2 and _rel(ref, w32.grad) < 1e-2
    assert _rel(acc, ref) < 1e-2


def test_conv1x1_xl_route_accumulates(monkeypatch):
    """Rows above the 4-wave TN threshold: gemm_tn_xl's split reduce adds."""
    from distributed_model_parallel_amd.ops import conv1x1 as c1
    from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1
    monkeypatch.setattr(c1, "_TN_XL_MIN_ROWS", 1024)
    torch.manual_seed(1)
    conv = Conv1x1(256, 256).to(DEV, torch.bfloat16).to(memory_format=CL)
    xs = [torch.randn(16, 256, 16, 16, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    gs = [torch.randn(16, 256, 16, 16, device=DEV).bfloat16() for _ in range(2)]
    before = c1._STATS["tn_xl"]

    def fn(i):
        conv(xs[i]).backward(gs[i])
    (acc,), used = _twice(fn, [conv.weight], True)
    assert used == 2 and c1._STATS["tn_xl"] - before == 2
    (ref,), _ = _twice(fn, [conv.weight], False)
    assert _rel(acc, ref) < 1e-2


@pytest.mark.parametrize("stride", [1, 2])
def test_depthwise_wgrad_accumulates_in_kernel(stride):
    from distributed_model_parallel_amd.ops.depthwise import DepthwiseConv2d
    torch.manual_seed(2)
    conv = DepthwiseConv2d(96, stride=stride).to(DEV, torch.bfloat16)
    xs = [torch.randn(8, 96, 16, 16, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    ho = (16 - 1) // stride + 1
    gs = [torch.randn(8, 96, ho, ho, device=DEV).bfloat16() for _ in range(2)]

    def fn(i):
        conv(xs[i]).backward(gs[i])
    (acc,), used = _twice(fn, [conv.weight], True)
    (ref,), _ = _twice(fn, [conv.weight], False)
    assert used == 2
    w32 = conv.weight.detach().float().requires_grad_()
    for i in range(2):
        F.conv2d(xs[i].float(), w32, None, stride, 1, 1, 96).backward(gs[i].float())
    assert _rel(acc, w32.grad) < 1e-2 and _rel(acc, ref) < 1e-2


@pytest.mark.parametrize("act,res", [("relu", False), (None, True)])
def test_bn_affine_grads_accumulate_in_kernel(act, res):
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(3)
    bn = BatchNormAct2d(64, act=act).to(DEV)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    xs = [torch.randn(8, 64, 8, 8, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    rs = [torch.randn(8, 64, 8, 8, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    gs = [torch.randn(8, 64, 8, 8, device=DEV).bfloat16() for _ in range(2)]

    def fn(i):
        bn(xs[i], rs[i] if res else None).backward(gs[i])
    (aw, ab), used = _twice(fn, [bn.weight, bn.bias], True)
    (rw, rb), _ = _twice(fn, [bn.weight, bn.bias], False)
    assert used == 4  # weight and bias, two micro-batches
    assert _rel(aw, rw) < 1e-5 and _rel(ab, rb) < 1e-5


def test_target_refuses_mismatched_grads():
    from distributed_model_parallel_amd.ops import grad_accum
    p = torch.nn.Parameter(torch.randn(16, 8, device=DEV).bfloat16())
    with grad_accum.accumulate_param_grads():
        assert grad_accum.target(p) is None  # no grad yet: autograd creates it
        p.grad = torch.zeros(8, 16, device=DEV).bfloat16().t()  # not dense row-major
        assert grad_accum.target(p) is None
        p.grad = torch.zeros_like(p)
        assert grad_accum.target(p) is p.grad
    assert grad_accum.target(p) is None  # mode off


@pytest.mark.parametrize("graphs", [False, True])
def test_pipeline_kernel_accumulation_matches_autograd(graphs):
    """MobileNetV2 bf16 stage, 1F1B over 4 micro-batches: the in-kernel
    accumulation gives the autograd engine's gradients (bf16 rounding apart),
    eager and on captured stage graphs."""
    import copy
    from distributed_model_parallel_amd.models import MobileNetV2
    from distributed_model_parallel_amd.ops import grad_accum
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    from tests.test_gpu_pipeline import _comm
    comm = _comm()
    torch.manual_seed(0)
    atoms = MobileNetV2(num_classes=10).as_sequential()
    pipes = [Pipeline(copy.deepcopy(atoms), comm, (3, 32, 32), micro_batches=4, schedule="1f1b",
                      device=torch.device("cuda", 0), dtype=torch.bfloat16, channels_last=True, static_batch=64,
                      graphs=graphs, kernel_grad_accum=k) for k in (False, True)]
    g = torch.Generator().manual_seed(1)
    x = torch.randn(64, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (64,), generator=g)
    from distributed_model_parallel_amd.ops import wt_cache
    before, hits = grad_accum.stats()["kernel"], wt_cache.stats()["hit"]
    res = [p.train_step(x, y) for p in pipes]
    assert grad_accum.stats()["kernel"] > before
    assert wt_cache.stats()["hit"] > hits  # the step's W^T buffers served the data gradients
    assert abs(float(res[0].loss) - float(res[1].loss)) < 1e-3 * max(1.0, float(res[0].loss))
    norms = sorted(float(p.grad.float().norm()) for p in pipes[0].module.parameters())
    floor = 1e-3 * norms[len(norms) // 2]
    for a, b in zip(pipes[0].module.parameters(), pipes[1].module.parameters()):
        err = float((a.grad.float() - b.grad.float()).norm())
        assert err <= 2e-2 * float(a.grad.float().norm()) + floor, (err, float(a.grad.float().norm()))


def test_conv1x1_strided_wgrad_on_tap_gather(monkeypatch):
    """Stride-2 1x1 weight gradients (the ResNet downsample) on the 4-wave TN
    kernel's tap gather (conv_wgrad_xl): fp32 reference, and accumulation."""
    from distributed_model_parallel_amd.ops import conv1x1 as c1
    from distributed_model_parallel_amd.ops.conv1x1 import Conv1x1
    monkeypatch.setattr(c1, "_TN_XL_MIN_ROWS", 1024)
    torch.manual_seed(5)
    conv = Conv1x1(256, 128, stride=2).to(DEV, torch.bfloat16).to(memory_format=CL)
    xs = [torch.randn(16, 256, 16, 16, device=DEV).bfloat16().contiguous(memory_format=CL) for _ in range(2)]
    gs = [torch.randn(16, 128, 8, 8, device=DEV).bfloat16() for _ in range(2)]
    before = c1._STATS["tn_xl_strided"]

    def fn(i):
        conv(xs[i]).backward(gs[i])
    (acc,), used = _twice(fn, [conv.weight], True)
    assert used == 2 and c1._STATS["tn_xl_strided"] - before == 2
    w32 = conv.weight.detach().float().requires_grad_()
    for i in range(2):
        F.conv2d(xs[i].float(), w32, None, 2).backward(gs[i].float())
    assert _rel(acc, w32.grad) < 1e-2
