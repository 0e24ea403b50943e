"""Optimizers: MasterSGD (fp32 master weights for any parameter list, used by
DP / pipeline / single-GPU training) must reproduce torch.optim.SGD in fp32 and
keep updates that bf16 SGD would drop (DP/pipe precision parity)."""
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
