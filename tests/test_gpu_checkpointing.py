"""Activation checkpointing on the native GPU path (bench/CLI
--checkpoint-segments): inside a checkpointed trunk the cross-layer fusions
(BN fold, BN+ReLU-in-GEMM, parked gradients) are off in BOTH the first
forward and the recompute (utils/checkpointing.in_checkpoint), so the
recompute rebuilds exactly the saved tensors of the first forward.  The
checkpointed ResNet-50 step must run and match the plain (fused) step to bf16
tolerance, with running statistics updated once."""
import copy

import pytest
import torch

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.ops.loss import cross_entropy
from distributed_model_parallel_amd.utils.checkpointing import enable_activation_checkpointing
from distributed_model_parallel_amd.utils.precision import cast_model

pytestmark = pytest.mark.gpu


def _grad_cos(a_mod, b_mod):
    dot = na = nb = 0.0
    for a, b in zip(a_mod.parameters(), b_mod.parameters()):
        a32, b32 = a.grad.float(), b.grad.float()
        dot += (a32 * b32).sum().item()
        na += a32.pow(2).sum().item()
        nb += b32.pow(2).sum().item()
    return dot / max((na * nb) ** 0.5, 1e-30)


def _grad_rel(a_mod, b_mod):
    num = den = 0.0
    for a, b in zip(a_mod.parameters(), b_mod.parameters()):
        num += (a.grad.float() - b.grad.float()).pow(2).sum().item()
        den += a.grad.float().pow(2).sum().item()
    return (num / max(den, 1e-30)) ** 0.5


@pytest.mark.parametrize("arch,size", [("resnet50", 64), ("mobilenetv2", 32)])
def test_checkpointed_step_matches_plain(arch, size, monkeypatch):
    """Reference: the same segments run WITHOUT recomputation but inside the
    checkpoint context (so the same unfused kernels run): the checkpointed
    step's recompute must rebuild the first forward's saved tensors exactly,
    so loss, gradients and running statistics match it to rounding.  The
    plain fused step is a looser sanity bound (different kernels; bf16 BN over
    8 images amplifies their rounding differences: 3 % in the loss, round 4)."""
    from distributed_model_parallel_amd.utils import checkpointing
    torch.manual_seed(0)
    m = build_model(arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    if arch == "resnet50":
        # tame the random-init residual branches (gamma 0.25 on each block's
        # last BN, between the stock 1 and zero_init_residual's 0): at gamma 1 the
        # 16 blocks amplify bf16 rounding so much at batch 8 that even the SAME
        # kernels in a different backward order land at gradient cosine 0.86-0.99
        # run to run (round 4), and both bf16 paths at 0.13 from fp32
        with torch.no_grad():
            for mod in m.modules():
                if hasattr(mod, "bn3"):
                    mod.bn3.weight.mul_(0.25)
    m0_state = {k: v.clone() for k, v in m.state_dict().items()}
    cast_model(m, torch.bfloat16)
    m2, m3 = copy.deepcopy(m), copy.deepcopy(m)
    enable_activation_checkpointing(m2, 4)
    enable_activation_checkpointing(m3, 4)
    x = torch.randn(8, 3, size, size, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.arange(8, device="cuda") % 10
    l1 = cross_entropy(m(x), y)
    l1.backward()
    l2 = cross_entropy(m2(x), y)
    l2.backward()

    def no_recompute(fn, *args, **kw):
        with checkpointing._flags(False):
            return fn(*args)
    monkeypatch.setattr(checkpointing, "checkpoint", no_recompute)
    l3 = cross_entropy(m3(x), y)
    l3.backward()
    monkeypatch.undo()
    # the forwards run the same kernels, but the BN moments' cross-block fp64
    # atomic adds land in a run-dependent order and bf16 BN over 8 images
    # amplifies that last-bit difference (round 4: 0.24 % in the loss once)
    torch.testing.assert_close(l2.float(), l3.float(), atol=1e-2, rtol=1e-2)
    # backward node ORDER differs (the recompute runs when a segment's first
    # saved tensor is unpacked), which changes where bf16 gradient sums round,
    # and the cross-block BN moment reduce adds in fp64 atomics (order varies
    # run to run); bf16 BN over 8 images amplifies both (round 4: 1.7 % and
    # 8.7 % in two runs) -- the gradient must still point the same way (with
    # the tamed residual branches: 0.97-0.99 over round-4 runs; a recompute that
    # rebuilt different activations or BN statistics falls far below)
    cos = _grad_cos(m3, m2)
    assert cos > 0.95, f"checkpointed vs same-kernel reference: gradient cosine {cos:.4f}"
    for (n, a), b in zip(m3.named_buffers(), m2.buffers()):
        if a.dtype.is_floating_point:
            # (1e-2: the forward's rare fp64-atomic-order rounding flips reach
            # layer 3's batch variance; a second running-stat update in the
            # recompute is caught exactly by num_batches_tracked below)
            torch.testing.assert_close(b.float(), a.float(), atol=1e-2, rtol=1e-2, msg=n)
        else:
            assert torch.equal(a, b), n  # num_batches_tracked: one update, not two
    torch.testing.assert_close(l2.float(), l1.float(), atol=0.1, rtol=0.1)
    # fused vs checkpointed (different kernels): judge each against an fp32
    # oracle of the same weights, relative to stock PyTorch bf16's own distance
    # from it: the checkpointed path no further than the fused
    # (MobileNetV2 at 32 px is not chaotic that way: fused ~ checkpointed > 0.9
    # directly; its stock fp32 channels-last backward aborted inside MIOpen on
    # the box once, so no oracle there)
    if arch != "resnet50":
        assert _grad_cos(m, m2) > 0.9
        return
    ref = build_model(arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    ref.load_state_dict({k: v.float() for k, v in m0_state.items()})
    with _native.reference_mode():
        cross_entropy(ref(x.float()), y).backward()
    # what bf16 itself costs here: stock PyTorch in bf16 on the same weights
    # (judge the native paths against that, not against a fixed 0.03;
    # tests/test_gpu_parity_train.py pins native == stock-bf16 distance in a
    # well-conditioned regime)
    sb = build_model(arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    sb.load_state_dict({k: v.float() for k, v in m0_state.items()})
    sb = sb.bfloat16()
    with _native.reference_mode():
        cross_entropy(sb(x).float(), y).backward()
    cf, cc, cb = _grad_cos(m, ref), _grad_cos(m2, ref), _grad_cos(sb, ref)
    print("gradient cosine to fp32: fused", cf, "checkpointed", cc, "stock bf16", cb)
    # round 5: fused 0.889, checkpointed 0.892, stock bf16 0.889
    assert cc > cb - 0.05 and cf > cb - 0.05, (cf, cc, cb)
