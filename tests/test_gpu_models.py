"""Whole-model check of the native path: a bf16 channels-last model (our MFMA
1x1 / implicit-GEMM / depthwise convs, fused BN kernels) against the same
weights in fp32 running plain PyTorch ops (the native kernels only take bf16,
so the fp32 copy is the reference).  Compares the loss and every parameter
gradient by cosine similarity and relative norm.

BatchNorm runs in eval mode (running statistics) here: with batch statistics
at these tiny test batches a random-init ResNet-50's gradients are chaotic --
measured with tools/noise_probe.py, a 1-ulp input perturbation alone drops the
median per-parameter gradient cosine to 0.18 and two MIOpen runs of the same
inputs agree only to 0.79 -- so a train-mode comparison cannot separate bugs
from rounding.  Train-mode BN numerics are covered per kernel
(test_gpu_kernels.py) and by the per-layer conv tests."""
import copy

import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.ops import conv1x1, conv_igemm, depthwise
from distributed_model_parallel_amd.utils.precision import cast_model

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _grads(model, x, y):
    model.zero_grad(set_to_none=True)
    loss = F.cross_entropy(model(x).float(), y)
    loss.backward()
    return loss.item(), {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}


@pytest.mark.parametrize("name,shape,ncls", [("resnet50", (8, 3, 64, 64), 1000),
                                             ("resnet18", (8, 3, 64, 64), 1000),
                                             ("mobilenetv2", (16, 3, 32, 32), 10)])
def test_native_model_grads_match_fp32(name, shape, ncls):
    torch.manual_seed(0)
    ref = build_model(name, num_classes=ncls).to(DEV).to(memory_format=torch.channels_last)
    nat = cast_model(copy.deepcopy(ref), torch.bfloat16)
    ref.eval()
    nat.eval()
    x = torch.randn(*shape, device=DEV).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (shape[0],), device=DEV)
    before = {k: d["native"] for k, d in (("1x1", conv1x1._STATS), ("ig", conv_igemm._STATS),
                                          ("dw", depthwise._STATS))}
    l_nat, g_nat = _grads(nat, x.bfloat16(), y)
    used = {k: d["native"] - before[k] for k, d in (("1x1", conv1x1._STATS), ("ig", conv_igemm._STATS),
                                                    ("dw", depthwise._STATS))}
    assert sum(used.values()) > 0, "native conv kernels were not used"
    l_ref, g_ref = _grads(ref, x, y)
    _compare(l_nat, g_nat, l_ref, g_ref)


def _compare(l_nat, g_nat, l_ref, g_ref, min_cos=0.95, median_cos=0.99):
    """Every parameter within min_cos (the stem conv, deepest in the backward
    chain, collects the most rounding), the median within median_cos."""
    assert abs(l_nat - l_ref) < 0.05 * max(1.0, abs(l_ref)), (l_nat, l_ref)
    bad, coss = [], []
    for n, gr in g_ref.items():
        gn = g_nat[n]
        if gr.norm() < 1e-6:
            continue
        cos = F.cosine_similarity(gn.flatten(), gr.flatten(), dim=0).item()
        rel = (gn.norm() / gr.norm()).item()
        coss.append(cos)
        if cos < min_cos or not 0.9 < rel < 1.1:
            bad.append(f"{n}: cos={cos:.4f} norm_ratio={rel:.3f}")
    assert not bad, "\n".join(bad)
    coss.sort()
    assert coss[len(coss) // 2] >= median_cos, f"median gradient cosine {coss[len(coss) // 2]:.4f}"


@pytest.mark.parametrize("name", ["resnet50", "resnet18"])
def test_igemm_vs_miopen_in_model(name):
    """Same bf16 model and data; only the 3x3 convs differ (implicit GEMM vs MIOpen)."""
    torch.manual_seed(0)
    m = cast_model(build_model(name, num_classes=100).to(DEV).to(memory_format=torch.channels_last))
    m.eval()
    x = torch.randn(32, 3, 64, 64, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (32,), device=DEV)
    state = copy.deepcopy(m.state_dict())
    n0 = conv_igemm._STATS["native"]
    l_a, g_a = _grads(m, x, y)
    assert conv_igemm._STATS["native"] > n0
    m.load_state_dict(state)
    conv_igemm.ENABLED = False
    try:
        l_b, g_b = _grads(m, x, y)
    finally:
        conv_igemm.ENABLED = True
    _compare(l_a, g_a, l_b, g_b, min_cos=0.97, median_cos=0.995)


@pytest.mark.parametrize("stride,ds", [(1, False), (2, True), (1, True)])
def test_bottleneck_fused_shortcut_grad(stride, ds):
    """conv1's dgrad epilogue absorbs the shortcut gradient (GradSlot): same x.grad
    as the unfused composition of the same modules (which adds in a separate kernel)."""
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    torch.manual_seed(0)
    cin, planes = (256, 64) if not ds else (128, 64)
    down = None
    if ds:
        down = torch.nn.Sequential(conv1x1.Conv1x1(cin, planes * 4, stride),
                                   __import__("distributed_model_parallel_amd.ops.batchnorm", fromlist=["x"]).BatchNormAct2d(planes * 4))
    blk = cast_model(Bottleneck(cin, planes, stride, down).to(DEV).to(memory_format=torch.channels_last))
    blk.train()
    x = torch.randn(8, cin, 16, 16, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    g = None
    outs = []
    from distributed_model_parallel_amd.ops import bn_fold
    fold_was = bn_fold.ENABLED
    for fused in (True, False):
        xi = x.detach().requires_grad_()
        n0 = conv1x1._STATS["fused_dgrad"]
        if fused:
            # isolate the shortcut fusion: bn3 unfolded (the fold has its own
            # fp32-referenced tests, tests/test_gpu_bn_fold.py)
            bn_fold.ENABLED = False
            try:
                y = blk(xi)
            finally:
                bn_fold.ENABLED = fold_was
        else:
            idn = xi if down is None else down[1](down[0](xi))
            out = blk.bn1(blk.conv1(xi))
            out = blk.bn2(blk.conv2(out))
            y = blk.bn3(blk.conv3(out), idn)
        if g is None:
            g = torch.randn_like(y)
        y.backward(g)
        if fused:
            assert conv1x1._STATS["fused_dgrad"] == n0 + 1, "shortcut gradient was not fused"
        outs.append(xi.grad.float())
    err = (outs[0] - outs[1]).norm() / outs[1].norm()
    assert err < 2e-2, err


@pytest.mark.parametrize("stride", [1, 2])
def test_bottleneck_bn_relu_fused_into_conv3(stride):
    """bn2's apply + ReLU inside conv3's GEMM (ops/fused.py bn_relu_conv1x1): same output,
    gradients and running statistics as the unfused composition of the same modules."""
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    from distributed_model_parallel_amd.ops import fused
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d
    torch.manual_seed(0)
    cin, planes = 256, 64
    down = None
    if stride != 1:
        down = torch.nn.Sequential(conv1x1.Conv1x1(cin, planes * 4, stride), BatchNormAct2d(planes * 4))
    from distributed_model_parallel_amd.models import resnet as resnet_mod
    old_flag, resnet_mod._FUSE_BN2_CONV3 = resnet_mod._FUSE_BN2_CONV3, True
    blk = cast_model(Bottleneck(cin, planes, stride, down).to(DEV).to(memory_format=torch.channels_last))
    with torch.no_grad():
        blk.bn3.weight.normal_(1.0, 0.1)  # not zero-init, so conv3's path matters
    ref = copy.deepcopy(blk)
    blk.train()
    ref.train()
    x = torch.randn(8, cin, 16, 16, device=DEV).bfloat16().contiguous(memory_format=torch.channels_last)
    xa, xb = x.detach().requires_grad_(), x.detach().requires_grad_()
    n0 = fused._STATS_FUSED["bn_relu_conv1x1"]
    try:
        ya = blk(xa)
    finally:
        resnet_mod._FUSE_BN2_CONV3 = old_flag
    assert fused._STATS_FUSED["bn_relu_conv1x1"] == n0 + 1
    idn = xb if down is None else ref.downsample[1](ref.downsample[0](xb))
    out = ref.bn1(ref.conv1(xb))
    out = ref.bn2(ref.conv2(out))
    yb = ref.bn3(ref.conv3(out), idn)
    torch.testing.assert_close(ya.float(), yb.float(), atol=5e-2, rtol=5e-2)
    g = torch.randn_like(ya)
    ya.backward(g)
    yb.backward(g)
    for (na, pa), (nb, pb) in zip(blk.named_parameters(), ref.named_parameters()):
        cos = F.cosine_similarity(pa.grad.float().flatten(), pb.grad.float().flatten(), dim=0).item()
        assert cos > 0.99, (na, cos)
    cos = F.cosine_similarity(xa.grad.float().flatten(), xb.grad.float().flatten(), dim=0).item()
    assert cos > 0.99, cos
    torch.testing.assert_close(blk.bn2.running_mean, ref.bn2.running_mean, atol=1e-3, rtol=1e-2)
    torch.testing.assert_close(blk.bn2.running_var, ref.bn2.running_var, atol=1e-3, rtol=1e-2)
    assert int(blk.bn2.num_batches_tracked) == int(ref.bn2.num_batches_tracked) == 1
