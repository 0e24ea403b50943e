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


@pytest.mark.parametrize("cout,cin,k", [(64, 64, 3), (256, 256, 3), (512, 128, 3), (96, 64, 5), (128, 128, 1)])
def test_multi_transpose_flipped_taps(cout, cin, k):
    """Tap-wise, flipped transposes: a channels-last [Cout, Cin, k, k] weight's
    storage [Cout, k*k*Cin] -> w.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, -1),
    mixed with plain transposes in one launch."""
    from distributed_model_parallel_amd import _native
    from distributed_model_parallel_amd.ops import wt_cache
    C = _native.require("multi_transpose")
    torch.manual_seed(1)
    w = torch.randn(cout, cin, k, k, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    p = torch.randn(300, 70, device="cuda").bfloat16()
    src = wt_cache._flip_src(w)
    d = torch.empty(cin, k * k * cout, device="cuda", dtype=torch.bfloat16)
    dp = torch.empty(70, 300, device="cuda", dtype=torch.bfloat16)
    dn = torch.empty(cin, k * k * cout, device="cuda", dtype=torch.bfloat16)
    C.multi_transpose([src, p, src], [d, dp, dn], [-k * k, 1, k * k])
    assert torch.equal(d, w.flip(2, 3).permute(1, 2, 3, 0).reshape(cin, -1))
    assert torch.equal(dn, w.permute(1, 2, 3, 0).reshape(cin, -1))
    assert torch.equal(dp, p.t())


def test_flipped_weights_cached_by_the_optimizer():
    """ResNet-50 bf16 + MasterSGD: after each optimizer step every cached
    flipped 3x3 weight equals the torch expression on the UPDATED weight, and
    the next backward reads it (hits).  (Whole-run weights are not compared
    bitwise: ResNet-50's fp64-atomic BN moment reduction is not bit-
    reproducible from run to run.)"""
    from distributed_model_parallel_amd.models import build_model
    from distributed_model_parallel_amd.ops import wt_cache
    from distributed_model_parallel_amd.ops.optim import MasterSGD
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(0)
    m = cast_model(build_model("resnet50", num_classes=10).cuda()).to(memory_format=torch.channels_last)
    x = torch.randn(32, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (32,), device="cuda")
    opt = MasterSGD(m.parameters(), lr=0.05, momentum=0.9)
    wt_cache.set_enabled(True)
    hits = []
    for i in range(3):
        h0 = wt_cache.stats()["hit"]
        loss = torch.nn.functional.cross_entropy(m(x).float(), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        hits.append(wt_cache.stats()["hit"] - h0)
        flips = {k: e for k, e in wt_cache._GLOBAL.items() if len(k) > 2 and k[2] == "flip"}
        assert flips, "no flipped weight entered the cache"
        for k, e in flips.items():
            w = e[0]()
            assert torch.equal(e[1], w.flip(2, 3).permute(1, 2, 3, 0).reshape(w.shape[1], -1))
        # the fp32 copies the BN-fold coefficient products read (ops/bn_fold.py)
        f32 = {k: e for k, e in wt_cache._GLOBAL.items() if len(k) > 2 and k[2] == "f32"}
        assert f32, "no fp32 weight copy entered the cache"
        for k, e in f32.items():
            w = e[0]()
            assert torch.equal(e[1], w.float().reshape(w.shape[0], -1))
    assert hits[-1] > hits[0], hits


def test_multi_cast_matches_torch():
    from distributed_model_parallel_amd import _native
    C = _native.require("multi_cast_bf16_f32")
    torch.manual_seed(2)
    srcs = [torch.randn(n, device="cuda").bfloat16() for n in (1, 7, 2048, 2049, 5000, 1 << 20)] * 12
    dsts = [torch.empty(s.numel(), device="cuda") for s in srcs]
    C.multi_cast_bf16_f32(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.float())
