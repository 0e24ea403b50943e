"""Convergence regression of the whole native training path.

The reference's only correctness claim is accuracy (MobileNetV2 CIFAR-10:
MP 93.3 % / DP 93.8 %, reference Readme.md:283-286, loop in
data_parallel.py:99-156).  CIFAR-10 is not available offline, so that number
stays unpinned; what IS checked here, on a fixed learnable synthetic task
(class-conditional templates + noise, CIFAR-shaped), is that the native stack
-- bf16 weights/activations, channels-last, fused BN forward/backward
(BnBwdSlot hand-offs, compact shortcut, stem-pool fusion), MFMA conv kernels,
halo 3x3 kernels, fused cross-entropy, the C++ DDP reducer and FlatSGD with
fp32 masters -- TRAINS like stock PyTorch: the same model object, the same
initial weights and the same batches, trained once natively and once in
``_native.reference_mode()`` (stock F.conv2d / F.batch_norm / torch SGD in
fp32).  The loss curves must stay inside a band and both runs must learn the
task.  Set DMP_CONVERGENCE_OUT=<file.json> to dump the curves.
"""
import copy
import json
import os
import subprocess
import sys
import tempfile

import pytest
import torch
import torch.nn.functional as F

from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.models import build_model

pytestmark = pytest.mark.gpu


def _task(n_cls, shape, n, seed=0, noise=2.0):
    g = torch.Generator().manual_seed(seed)
    c, h, w = shape
    # low-frequency class templates (upsampled 8x8 noise): learnable, not trivial
    t = torch.randn(n_cls, c, 8, 8, generator=g)
    t = F.interpolate(t, size=(h, w), mode="bilinear", align_corners=False)
    t = t / t.std(dim=(1, 2, 3), keepdim=True)
    y = torch.randint(0, n_cls, (n,), generator=g)
    x = t[y] + noise * torch.randn(n, c, h, w, generator=g)
    return x, y


WARMUP = 30


def _lr(lr, i):
    """Linear warm-up (the reference recipe's) for both runs: without
    it a random-init ResNet-50's first ~20 steps are chaotic -- measured, loss
    excursions to 5-9 whose size differs run to run even for two stock fp32
    runs -- and windowed comparisons in that phase test the chaos, not the kernels."""
    return lr * min(1.0, (i + 1) / WARMUP)


def _ensure_pg():
    import torch.distributed as dist
    if not dist.is_initialized():  # one rank: an in-process store, no TCP port to race for
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)


@pytest.fixture(scope="module", autouse=True)
def _destroy_pg():
    yield
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def _train_native(model, xs, ys, steps, batch, lr):
    from distributed_model_parallel_amd.ops.loss import cross_entropy
    from distributed_model_parallel_amd.ops.optim import FlatSGD
    from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
    from distributed_model_parallel_amd.utils.precision import cast_model
    _ensure_pg()
    m = model.cuda().to(memory_format=torch.channels_last)
    cast_model(m, torch.bfloat16)
    ddp = DistributedDataParallel(m, flat_parameters=True)
    opt = FlatSGD(ddp, lr=lr, momentum=0.9, weight_decay=5e-4)
    losses = []
    for i in range(steps):
        for g in opt.param_groups:
            g["lr"] = _lr(lr, i)
        sl = slice((i * batch) % xs.shape[0], (i * batch) % xs.shape[0] + batch)
        x = xs[sl].cuda().bfloat16().contiguous(memory_format=torch.channels_last)
        y = ys[sl].cuda()
        loss = cross_entropy(ddp(x), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.detach().float())
    return m, [float(v) for v in torch.stack(losses).cpu()]


def _train_reference(model, xs, ys, steps, batch, lr):
    m = model.cuda()
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    losses = []
    with _native.reference_mode():
        for i in range(steps):
            for g in opt.param_groups:
                g["lr"] = _lr(lr, i)
            sl = slice((i * batch) % xs.shape[0], (i * batch) % xs.shape[0] + batch)
            loss = F.cross_entropy(m(xs[sl].cuda()), ys[sl].cuda())
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.detach())
    return m, [float(v) for v in torch.stack(losses).cpu()]


@torch.no_grad()
def _accuracy(m, x, y, native, batch=256):
    m.eval()
    ok = 0
    ctx = _native.reference_mode() if not native else torch.no_grad()
    with ctx:
        for i in range(0, x.shape[0], batch):
            xb = x[i:i + batch].cuda()
            if native:
                xb = xb.bfloat16().contiguous(memory_format=torch.channels_last)
            ok += (m(xb).float().argmax(1).cpu() == y[i:i + batch]).sum().item()
    m.train()
    return 100.0 * ok / x.shape[0]


def _mean(v):
    return sum(v) / len(v)


# The stock fp32 reference trains in a CHILD process: a fresh process holds
# none of the earlier GPU tests' state.  (Run inside the suite, the reference
# backward aborted -- SIGABRT in the autograd device thread, message lost to
# pytest's capture -- in 2 of 4 full-suite runs of one build, never when this
# file ran alone: profiles/README.md finding 77.  An abort here took the whole
# suite down; a failing child fails only this test.)
_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reference_in_child(kind, model, arch, ncls, steps, batch, lr, **data):
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "ref.pt")
        torch.save(dict(kind=kind, arch=arch, ncls=ncls, steps=steps, batch=batch, lr=lr,
                        state={k: v.detach().cpu() for k, v in model.state_dict().items()}, **data), path)
        code = ("import sys; sys.path.insert(0, %r); import importlib.util as u; "
                "s = u.spec_from_file_location('conv_child', %r); m = u.module_from_spec(s); "
                "s.loader.exec_module(m); m._child_main(%r)") % (_ROOT, os.path.abspath(__file__), path)
        r = subprocess.run([sys.executable, "-c", code], cwd=_ROOT, capture_output=True, text=True, timeout=1500)
        assert r.returncode == 0, f"reference child rc={r.returncode}\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
        with open(path + ".json") as f:
            return json.load(f)


def _child_main(path):
    p = torch.load(path, weights_only=True)
    m = build_model(p["arch"], num_classes=p["ncls"])
    m.load_state_dict(p["state"])
    out = {}
    if p["kind"] == "small":
        ref, out["losses"] = _train_reference(m, p["xs"], p["ys"], p["steps"], p["batch"], p["lr"])
        out["acc"] = _accuracy(ref, p["xh"], p["yh"], False)
    else:
        data = _Templates(p["ncls"], p["size"], noise=p["noise"])
        out["losses"] = _train_reference_fn(m, data, p["steps"], p["batch"], p["lr"])
    with open(path + ".json", "w") as f:
        json.dump(out, f)


def _steps_to(v, thr, k=5):
    """First step whose k-step mean is below thr (None if never)."""
    for i in range(len(v) - k + 1):
        if _mean(v[i:i + k]) < thr:
            return i
    return None


@pytest.mark.parametrize("arch,shape,ncls,steps,batch,lr,noise", [
    ("mobilenetv2", (3, 32, 32), 10, 240, 128, 0.05, 6.0),
    # random-init ResNet-50 without warm-up diverges at lr 0.05 (stock and native alike)
    ("resnet50", (3, 64, 64), 10, 150, 128, 0.01, 3.0),
])
def test_native_training_tracks_stock_pytorch(arch, shape, ncls, steps, batch, lr, noise):
    torch.manual_seed(0)
    xs, ys = _task(ncls, shape, 8192, seed=1, noise=noise)
    gv = torch.Generator().manual_seed(7)
    base = build_model(arch, num_classes=ncls)
    ref0 = copy.deepcopy(base)
    nat, l_nat = _train_native(base, xs, ys, steps, batch, lr)
    # held-out samples: the same class templates (seed 1), labels and noise re-drawn
    xh, yh = _task(ncls, shape, 9216, seed=1, noise=noise)
    xh, yh = xh[8192:], yh[8192:]
    xh = xh + 0.25 * torch.randn(xh.shape, generator=gv)
    acc_nat = _accuracy(nat, xh, yh, True)
    r = _reference_in_child("small", ref0, arch, ncls, steps, batch, lr, xs=xs, ys=ys, xh=xh, yh=yh)
    l_ref, acc_ref = r["losses"], r["acc"]
    out = os.environ.get("DMP_CONVERGENCE_OUT")
    if out:
        rec = {}
        if os.path.exists(out):
            with open(out) as f:
                rec = json.load(f)
        rec[arch] = {"native_bf16": l_nat, "stock_fp32": l_ref, "acc_native": acc_nat, "acc_stock": acc_ref,
                     "steps": steps, "batch": batch, "lr": lr, "noise": noise, "shape": list(shape)}
        with open(out, "w") as f:
            json.dump(rec, f)
    k = max(10, steps // 6)
    # both learn the task (chance = 10 %)
    assert _mean(l_nat[-k:]) < 0.5 * _mean(l_nat[:k]), (l_nat[:5], l_nat[-5:])
    assert acc_ref > 80.0 and acc_nat > 80.0, (acc_nat, acc_ref)
    assert acc_nat > acc_ref - 10.0, (acc_nat, acc_ref)
    # the native curve never lags the stock one: the step at which the 5-step
    # mean first falls below 50 / 25 / 10 % of the initial loss is at most 25 %
    # (+8 steps) later than stock's.  Steps-to-threshold, not windowed means: in
    # the steep part of the curve a run that is a few steps ahead differs by
    # 1.5-2x in a window (measured, full-suite runs: MobileNetV2 steps 40-79
    # native 0.49 vs stock 0.34 one run, 0.49 vs 0.48 another), while a
    # lost / scaled gradient or a broken kernel needs ~2x the steps.
    l0 = _mean(l_ref[:5])
    for frac in (0.5, 0.25, 0.1):
        sn, sr = _steps_to(l_nat, frac * l0), _steps_to(l_ref, frac * l0)
        assert sr is not None and sn is not None and sn <= 1.25 * sr + 8, (frac, sn, sr)
    # and both end on the same plateau
    a, b = _mean(l_nat[-k:]), _mean(l_ref[-k:])
    assert abs(a - b) <= 0.25 * max(a, b) + 0.05, (a, b)


class _Templates:
    """A harder, 224-px task: ``ncls`` low-frequency class templates plus heavy
    noise, batches drawn deterministically per step (both runs see the same
    data), so the loss plateaus well above zero within the run and a subtly
    wrong gradient shows as a slower / higher curve."""

    def __init__(self, ncls, size, noise, seed=3):
        g = torch.Generator().manual_seed(seed)
        t = torch.randn(ncls, 3, 8, 8, generator=g)
        t = F.interpolate(t, size=(size, size), mode="bilinear", align_corners=False)
        self.t = t / t.std(dim=(1, 2, 3), keepdim=True)
        self.ncls, self.noise, self.seed = ncls, noise, seed

    def batch(self, i, n):
        g = torch.Generator().manual_seed(self.seed * 100003 + i)
        y = torch.randint(0, self.ncls, (n,), generator=g)
        return self.t[y] + self.noise * torch.randn(n, *self.t.shape[1:], generator=g), y


def _train_native_fn(model, data, steps, batch, lr):
    from distributed_model_parallel_amd.ops.loss import cross_entropy
    from distributed_model_parallel_amd.ops.optim import FlatSGD
    from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
    from distributed_model_parallel_amd.utils.precision import cast_model
    _ensure_pg()
    m = model.cuda().to(memory_format=torch.channels_last)
    cast_model(m, torch.bfloat16)
    ddp = DistributedDataParallel(m, flat_parameters=True)
    opt = FlatSGD(ddp, lr=lr, momentum=0.9, weight_decay=5e-4)
    losses = []
    for i in range(steps):
        for g in opt.param_groups:
            g["lr"] = _lr(lr, i)
        x, y = data.batch(i, batch)
        loss = cross_entropy(ddp(x.cuda().bfloat16().contiguous(memory_format=torch.channels_last)), y.cuda())
        loss.backward()
        opt.step()
        opt.zero_grad()
        losses.append(loss.detach().float())
    return [float(v) for v in torch.stack(losses).cpu()]


def _train_reference_fn(model, data, steps, batch, lr):
    m = model.cuda()
    opt = torch.optim.SGD(m.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    losses = []
    with _native.reference_mode():
        for i in range(steps):
            for g in opt.param_groups:
                g["lr"] = _lr(lr, i)
            x, y = data.batch(i, batch)
            loss = F.cross_entropy(m(x.cuda()), y.cuda())
            opt.zero_grad()
            loss.backward()
            opt.step()
            losses.append(loss.detach())
    return [float(v) for v in torch.stack(losses).cpu()]


def _bench_routes(steps=2):
    """The kernel routes of the headline bench step (bench.py defaults:
    ResNet-50, DDP, bf16, channels-last, 2048 images, 224 px)."""
    from distributed_model_parallel_amd.train.step import StepConfig, build_train_state
    from distributed_model_parallel_amd.utils import routes
    st = build_train_state(StepConfig(model="resnet50", batch_size=2048), torch.device("cuda", 0))
    st.step()
    r0 = routes.route_counts()
    for _ in range(steps):
        st.step()
    torch.cuda.synchronize()
    out = routes.active(routes.diff(routes.route_counts(), r0))
    del st
    torch.cuda.empty_cache()
    return out


def test_resnet50_224_training_covers_bench_routes_and_tracks_stock():
    """ResNet-50 at 224 px (the bench's kernel routing:
    stem_halo, halo c64/c128 forward / dgrad / wgrad, stride-phase dgrads,
    the BN fold with and without the downsample), on a task that does not
    saturate.  Every route the bench's timed steps take must also have run in
    this training run, and the native bf16 curve must track stock fp32."""
    from distributed_model_parallel_amd.utils import routes
    steps, batch, lr, ncls = 160, 64, 0.02, 100
    data = _Templates(ncls, 224, noise=4.0)
    torch.manual_seed(0)
    base = build_model("resnet50", num_classes=ncls)
    ref0 = copy.deepcopy(base)
    r0 = routes.route_counts()
    # the bench's batch-2048 weight gradients of layer 3 take the ping-pong TN
    # route (M >= 150k rows); train through it at batch 64 as well
    from distributed_model_parallel_amd.ops import conv1x1
    tn_min, conv1x1._TN_XL_MIN_ROWS = conv1x1._TN_XL_MIN_ROWS, 0
    try:
        l_nat = _train_native_fn(base, data, steps, batch, lr)
    finally:
        conv1x1._TN_XL_MIN_ROWS = tn_min
    trained = routes.active(routes.diff(routes.route_counts(), r0))
    del base
    torch.cuda.empty_cache()
    l_ref = _reference_in_child("t224", ref0, "resnet50", ncls, steps, batch, lr, size=224, noise=4.0)["losses"]
    del ref0
    torch.cuda.empty_cache()
    bench = _bench_routes()
    out = os.environ.get("DMP_CONVERGENCE_OUT")
    if out:
        rec = {}
        if os.path.exists(out):
            with open(out) as f:
                rec = json.load(f)
        rec["resnet50_224"] = {"native_bf16": l_nat, "stock_fp32": l_ref, "steps": steps, "batch": batch, "lr": lr,
                               "classes": ncls, "noise": 4.0, "routes_trained": trained, "routes_bench": bench}
        with open(out, "w") as f:
            json.dump(rec, f)
    miss = routes.missing(bench, trained)
    assert not miss, f"bench kernel routes never trained here: {miss}"
    k = 20
    l0 = _mean(l_ref[:5])
    a, b = _mean(l_nat[-k:]), _mean(l_ref[-k:])
    # the task is learned by the reference.  (Round 4 also required its plateau
    # to stay above 0.1 x start; a round-5 stock fp32 run ended at 0.087 x --
    # the stock curve's late value is as chaotic as the native one, and the
    # comparisons below do not need an unsaturated plateau.  Gradient parity
    # itself is pinned by tests/test_gpu_parity_train.py.)
    assert b < 0.9 * l0, (l0, b)
    # native tracks stock.  Before the descent sets in the two runs are
    # near-deterministic: over steps 0-29 the native / stock mean loss ratio
    # measured 1.001-1.018 per 10-step window (round 5, profiles/README.md
    # finding 66) -- a wrong gradient shows here first, so this is the tight
    # check.  From the descent's onset on the curves are separate trajectories
    # of a chaotic run: three round-5 runs of the SAME stock fp32 code put its
    # whole-curve mean at 3.03, 3.33 and 3.73 (native 3.44-3.95), so the
    # whole-curve ratio (measured 0.86-1.31) gets a band of that width, and a
    # real descent is required.  (Round 4's steps-to-95 / 90 % lag check is
    # dropped: the onset is the most chaotic part of the curve.)
    early_n, early_r = _mean(l_nat[:30]), _mean(l_ref[:30])
    assert abs(early_n / early_r - 1.0) <= 0.05, (early_n, early_r)
    assert _mean(l_nat) <= 1.4 * _mean(l_ref), (_mean(l_nat), _mean(l_ref))
    assert a < 0.6 * l0, (l0, a)
    # the descent itself is still checked, at bands wide enough for its chaos
    # (ADVICE r5): every 10-step window of steps 30-80 within 2x of stock, and
    # the native run reaching 90 % of the start loss (10-step running mean) no
    # later than 2 x stock's step + 15
    for w0 in range(30, min(80, len(l_nat), len(l_ref)) - 9, 10):
        wn, wr = _mean(l_nat[w0:w0 + 10]), _mean(l_ref[w0:w0 + 10])
        assert 0.5 <= wn / wr <= 2.0, (w0, wn, wr)

    def first_below(ls, frac):
        for i in range(len(ls) - 9):
            if _mean(ls[i:i + 10]) < frac * l0:
                return i
        return len(ls)
    sn, sr = first_below(l_nat, 0.9), first_below(l_ref, 0.9)
    assert sn <= 2 * sr + 15, (sn, sr)
