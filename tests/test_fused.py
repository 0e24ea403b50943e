"""GradSlot / grad_tap handshake (ops/fused.py): the shortcut gradient is either
absorbed by the consumer's backward or returned to autograd -- never lost or
double counted -- whatever order the engine runs the two nodes in."""
import torch

from distributed_model_parallel_amd.ops.fused import GradSlot, grad_tap


class _Consumer(torch.autograd.Function):
    """Stands in for the native 1x1 conv: y = 2x, dx = 2*dy (+ parked grad)."""

    @staticmethod
    def forward(ctx, x, slot):
        ctx.slot = slot
        slot.consumer = True
        return x * 2

    @staticmethod
    def backward(ctx, g):
        extra = ctx.slot.take()
        return (g * 2 if extra is None else g * 2 + extra), None


def _expected(x):
    return 2 + 18 * x


def test_tap_after_consumer_fuses():
    x = torch.randn(7, requires_grad=True)
    slot = GradSlot()
    a = _Consumer.apply(x, slot)
    b = grad_tap(x, slot) * 3          # created after the consumer -> runs first
    (a.sum() + (b * b).sum()).backward()
    torch.testing.assert_close(x.grad, _expected(x.detach()))
    assert not slot.consumer_ran  # the consumer absorbed the parked gradient


def test_tap_before_consumer_falls_back():
    x = torch.randn(7, requires_grad=True)
    slot = GradSlot()
    slot.consumer = True              # registered, but the consumer node is newer
    b = grad_tap(x, slot) * 3
    a = _Consumer.apply(x * 1.0, slot)
    (a.sum() + (b * b).sum()).backward()
    torch.testing.assert_close(x.grad, _expected(x.detach()))


def test_no_consumer_is_passthrough():
    x = torch.randn(7, requires_grad=True)
    slot = GradSlot()
    y = grad_tap(x, slot)
    assert y is x
    (y * 3).sum().backward()
    torch.testing.assert_close(x.grad, torch.full_like(x, 3.0))


def test_bottleneck_cpu_grads_unchanged():
    """The Bottleneck wiring (fallback path on CPU) matches a hand-built reference."""
    from distributed_model_parallel_amd.models.resnet import Bottleneck
    import copy
    torch.manual_seed(0)
    ds = torch.nn.Sequential(torch.nn.Conv2d(16, 32, 1, bias=False), torch.nn.BatchNorm2d(32))
    blk = Bottleneck(16, 8, 1, ds)
    ref = copy.deepcopy(blk)
    x = torch.randn(2, 16, 6, 6, requires_grad=True)
    xr = x.detach().clone().requires_grad_()
    blk(x).square().sum().backward()
    idn = ref.downsample(xr)
    out = ref.bn1(ref.conv1(xr))
    out = ref.bn2(ref.conv2(out))
    ref.bn3(ref.conv3(out), idn).square().sum().backward()
    torch.testing.assert_close(x.grad, xr.grad)
