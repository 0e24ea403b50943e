"""Optimizers: MasterSGD (fp32 master weights for any parameter list, used by
DP / pipeline / single-GPU training) must reproduce torch.optim.SGD in fp32 and
keep updates that bf16 SGD would drop (DP/pipe precision parity)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_model_parallel_amd.ops.optim import MasterSGD


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(),
                         nn.AdaptiveAvgPool2d(2), nn.Flatten(), nn.Linear(32, 5))


def test_master_sgd_matches_torch_sgd_fp32():
    a, b = _net(), _net()
    b = b.to(memory_format=torch.channels_last)
    oa = torch.optim.SGD(a.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    ob = MasterSGD(b.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    g = torch.Generator().manual_seed(1)
    for _ in range(3):
        x = torch.randn(4, 3, 6, 6, generator=g)
        y = torch.randint(0, 5, (4,), generator=g)
        for m, o in ((a, oa), (b, ob)):
            o.zero_grad()
            F.cross_entropy(m(x), y).backward()
            o.step()
    for (k, va), vb in zip(a.state_dict().items(), b.state_dict().values()):
        torch.testing.assert_close(va, vb, atol=1e-6, rtol=1e-5, msg=k)
    # parameters are views of one flat buffer, grads views of another
    st = ob._groups[0]
    assert all(p.grad.data_ptr() >= st["grad"].data_ptr() for p in b.parameters())


def test_master_sgd_keeps_sub_ulp_bf16_updates():
    p = nn.Parameter(torch.ones(16, dtype=torch.bfloat16))
    q = nn.Parameter(torch.ones(16, dtype=torch.bfloat16))
    om = MasterSGD([p], lr=1.0)
    ot = torch.optim.SGD([q], lr=1.0)
    for _ in range(10):
        for t, o in ((p, om), (q, ot)):
            o.zero_grad()
            (t.float() * 1e-3).sum().backward()  # lr*g = 1e-3 < half a bf16 ulp at 1.0
            o.step()
    assert torch.all(q == 1.0), "plain bf16 SGD drops the update (what MasterSGD fixes)"
    torch.testing.assert_close(om._groups[0]["master"][:16], torch.full((16,), 0.99))
    assert torch.all(p < 1.0)


def test_master_sgd_adopts_replaced_grads_and_state_roundtrip():
    m = _net()
    o = MasterSGD(m.parameters(), lr=0.1, momentum=0.9)
    F.cross_entropy(m(torch.randn(2, 3, 6, 6)), torch.tensor([0, 1])).backward()
    m[0].weight.grad = torch.ones_like(m[0].weight)  # replaced behind the optimizer's back
    m[5].bias.grad = None
    o.step()
    sd = o.state_dict()
    m2 = _net()
    o2 = MasterSGD(m2.parameters(), lr=0.1, momentum=0.9)
    o2.load_state_dict(sd)
    torch.testing.assert_close(o2._groups[0]["momentum"], o._groups[0]["momentum"])
    assert o2._steps == 1


def test_master_sgd_follows_weights_loaded_without_optimizer_state(tmp_path):
    """a checkpoint carrying only 'net' (the reference's
    {'net','acc','epoch'} format) loaded after MasterSGD exists must not be
    overwritten by the construction-time fp32 master on the first step."""
    from distributed_model_parallel_amd.utils.checkpoint import load_checkpoint
    src = _net().to(torch.bfloat16)
    with torch.no_grad():
        for p in src.parameters():
            p.add_(1.0)  # clearly different from _net()'s init
    path = str(tmp_path / "ckpt.pth")
    torch.save({"net": src.state_dict(), "acc": 50.0, "epoch": 3}, path)
    dst = _net().to(torch.bfloat16)
    opt = MasterSGD(dst.parameters(), lr=0.1, momentum=0.9, weight_decay=0.0)
    meta = load_checkpoint(path, dst, opt, restore_rng=False)
    assert meta["epoch"] == 3
    opt.zero_grad()
    opt.step()  # zero gradient, no weight decay: weights must stay the loaded ones
    for (k, a), b in zip(src.state_dict().items(), dst.state_dict().values()):
        assert torch.equal(a, b), k


def test_master_sgd_rejects_foreign_optimizer_state(tmp_path):
    """An older checkpoint holding a torch.optim.SGD state: warn, start fresh
    from the loaded weights instead of raising KeyError('numels')."""
    import warnings
    from distributed_model_parallel_amd.utils.checkpoint import load_checkpoint
    src = _net().to(torch.bfloat16)
    with torch.no_grad():
        for p in src.parameters():
            p.mul_(0.5)
    sgd = torch.optim.SGD(src.parameters(), lr=0.1, momentum=0.9)
    path = str(tmp_path / "ckpt.pth")
    torch.save({"net": src.state_dict(), "optimizer": sgd.state_dict(), "acc": 1.0, "epoch": 1}, path)
    dst = _net().to(torch.bfloat16)
    opt = MasterSGD(dst.parameters(), lr=0.1, momentum=0.0, weight_decay=0.0)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        load_checkpoint(path, dst, opt, restore_rng=False)
    assert any("optimizer state not restored" in str(x.message) for x in w)
    opt.zero_grad()
    opt.step()
    for a, b in zip(src.state_dict().values(), dst.state_dict().values()):
        assert torch.equal(a, b)


def test_master_sgd_layout_mismatch_is_an_error(tmp_path):
    """only a FOREIGN optimizer state is tolerated; a MasterSGD
    state whose parameter layout differs from the model must not be skipped
    silently (the resume would continue with fresh momentum)."""
    import pytest
    from distributed_model_parallel_amd.utils.checkpoint import load_checkpoint, save_checkpoint
    src = _net()
    opt_src = MasterSGD(src.parameters(), lr=0.1, momentum=0.9)
    path = save_checkpoint(str(tmp_path / "ck.pth"), src, opt_src, epoch=1)
    dst = _net()
    opt = MasterSGD(list(dst.parameters())[:-1], lr=0.1, momentum=0.9)  # one parameter short
    with pytest.raises(ValueError, match="layout differs"):
        load_checkpoint(path, dst, opt, restore_rng=False)


def test_checkpoint_with_legacy_numpy_rng_state_loads(tmp_path):
    """files whose RNG entry is np.random.get_state() (an
    ndarray) still load weights-only, and the numpy RNG is restored."""
    import numpy as np
    from distributed_model_parallel_amd.utils.checkpoint import load_checkpoint
    net = _net()
    np.random.seed(7)
    legacy = np.random.get_state()
    expect = np.random.rand(3)
    path = str(tmp_path / "legacy.pth")
    import random
    torch.save({"net": net.state_dict(), "acc": 0.0, "epoch": 0,
                "rng": {"python": random.getstate(), "numpy": legacy, "torch": torch.get_rng_state()}}, path)
    np.random.seed(99)
    load_checkpoint(path, _net(), restore_rng=True)
    assert np.allclose(np.random.rand(3), expect)


def test_schedule_resume_across_kinds_and_milestones():
    """a cosine checkpoint resumed with --lr-steps must not KeyError
    (the command line's milestones stay); different milestones / schedule
    kinds warn; a multistep checkpoint resumes its own milestones."""
    import warnings
    from distributed_model_parallel_amd.utils.schedule import build_schedule
    p = nn.Parameter(torch.zeros(1))
    cos = build_schedule(torch.optim.SGD([p], lr=0.4), 90, 5)
    cos.step(); cos.step()
    sd_cos = cos.state_dict()
    ms = build_schedule(torch.optim.SGD([p], lr=0.4), 90, 5, lr_steps=[30, 60])
    with pytest.warns(UserWarning, match="cosine"):
        ms.load_state_dict(sd_cos)
    assert ms.milestones == [30, 60] and ms.epoch == 2
    ms2 = build_schedule(torch.optim.SGD([p], lr=0.4), 90, 5, lr_steps=[10, 20])
    with pytest.warns(UserWarning, match="milestones"):
        ms2.load_state_dict(ms.state_dict())
    assert ms2.milestones == [30, 60]
    ms3 = build_schedule(torch.optim.SGD([p], lr=0.4), 90, 5, lr_steps=[30, 60])
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        ms3.load_state_dict(ms.state_dict())  # identical: silent
    cos2 = build_schedule(torch.optim.SGD([p], lr=0.4), 90, 5)
    with pytest.warns(UserWarning, match="multistep"):
        cos2.load_state_dict(ms.state_dict())
