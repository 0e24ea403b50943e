"""W^T of the 1x1-conv data gradients from the optimizer-driven cache
(ops/wt_cache.py) and the batched transpose kernel behind it."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shapes", [[(64, 64)], [(256, 64), (64, 1000), (7, 130), (2048, 512)] * 20])
def test_multi_transpose_matches_torch(shapes):
    from distributed_model_parallel_amd import _native
    C = _native.require("multi_transpose")
    torch.manual_seed(0)
    srcs = [torch.randn(r, c, device="cuda").bfloat16() for r, c in shapes]
    dsts = [torch.empty(c, r, device="cuda", dtype=torch.bfloat16) for r, c in shapes]
    C.multi_transpose(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.t())


def test_training_with_cached_wt_matches_uncached():
    """MobileNetV2 bf16 + MasterSGD for 4 steps: the cached W^T (refreshed by
    the optimizer) gives the same weights as a fresh transpose per backward."""
    from distributed_model_parallel_amd.models import MobileNetV2
    from distributed_model_parallel_amd.ops import wt_cache
    from distributed_model_parallel_amd.ops.optim import MasterSGD
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(0)
    base = cast_model(MobileNetV2(num_classes=10).cuda()).to(memory_format=torch.channels_last)
    x = torch.randn(64, 3, 32, 32, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (64,), device="cuda")
    out = []
    try:
        for on in (False, True):
            wt_cache.set_enabled(on)
            m = copy.deepcopy(base)
            opt = MasterSGD(m.parameters(), lr=0.05, momentum=0.9)
            h0 = wt_cache.stats()["hit"]
            for _ in range(4):
                loss = torch.nn.functional.cross_entropy(m(x).float(), y)
                loss.backward()
                opt.step()
                opt.zero_grad()
            hits = wt_cache.stats()["hit"] - h0
            assert (hits > 0) == on, hits
            out.append([p.detach().float().clone() for p in m.parameters()])
    finally:
        wt_cache.set_enabled(True)
    for a, b in zip(*out):
        assert torch.allclose(a, b, atol=1e-6, rtol=1e-5), float((a - b).abs().max())
