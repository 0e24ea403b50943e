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

from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.ops.loss import cross_entropy
from distributed_model_parallel_amd.utils.checkpointing import enable_activation_checkpointing
from distributed_model_parallel_amd.utils.precision import cast_model

pytestmark = pytest.mark.gpu


@pytest.mark.unvalidated
@pytest.mark.parametrize("arch,size", [("resnet50", 64), ("mobilenetv2", 32)])
def test_checkpointed_step_matches_plain(arch, size):
    torch.manual_seed(0)
    m = build_model(arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_model(m, torch.bfloat16)
    m2 = copy.deepcopy(m)
    enable_activation_checkpointing(m2, 4)
    x = torch.randn(8, 3, size, size, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.arange(8, device="cuda") % 10
    l1 = cross_entropy(m(x), y)
    l1.backward()
    l2 = cross_entropy(m2(x), y)
    l2.backward()
    torch.testing.assert_close(l2.float(), l1.float(), atol=2e-2, rtol=2e-2)
    num = den = 0.0
    for a, b in zip(m.parameters(), m2.parameters()):
        num += (a.grad.float() - b.grad.float()).pow(2).sum().item()
        den += a.grad.float().pow(2).sum().item()
    assert (num / max(den, 1e-30)) ** 0.5 < 0.05, f"relative grad error {(num / den) ** 0.5:.3g}"
    for (n, a), b in zip(m.named_buffers(), m2.buffers()):
        if a.dtype.is_floating_point:
            torch.testing.assert_close(a.float(), b.float(), atol=2e-2, rtol=2e-2, msg=n)
        else:
            assert torch.equal(a, b), n  # num_batches_tracked: one update, not two
