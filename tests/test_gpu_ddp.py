"""The RCCL path of DDP / SyncBN on one MI355X (world size 1, so no peers): the
reducer is forced onto the RCCL backend (ncclAllReduce avg over one rank) and
must give the same parameters after a training step as the no-op world-1
backend; SyncBatchNorm's moment all-reduce goes through RCCL too.  Runs in a
subprocess because the process group is process-global."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, torch
sys.path.insert(0, os.environ["ROOT"])
from distributed_model_parallel_amd.utils.env import init_distributed, destroy_distributed
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state
env = init_distributed()
out = {}
# resnet50: the BN fold (ops/bn_fold.py) routes its folded moments and backward
# sums through SyncBN's reducers -- RCCL all-reduces when forced
CASES = [("resnet18", "ddp"), ("resnet18", "syncbn"), ("resnet50", "syncbn")]
# one throwaway step per model first: MIOpen's find mode may pick another
# algorithm on a shape's first use (same as the ordering test below), and a
# random-init ResNet-50 with batch-statistics BN at batch 8 turns that rounding
# difference into ~0.5 % of the first loss
for model in sorted({m for m, _ in CASES}):
    build_train_state(StepConfig(model=model, batch_size=8, image_size=64, parallel="ddp"), env.device).step()
for model, parallel in CASES:
    for forced in ("0", "1"):
        os.environ["DMP_DDP_SINGLE_RANK_COMM"] = forced
        cfg = StepConfig(model=model, batch_size=8, image_size=64, parallel=parallel)
        st = build_train_state(cfg, env.device)
        before = [p.detach().float().clone() for p in st.model.parameters()]
        loss = st.step()          # one step: the update carries the (averaged) gradient
        torch.cuda.synchronize()
        delta = [p.detach().float() - b for p, b in zip(st.model.parameters(), before)]
        out[(model, parallel, forced)] = (loss.item(), delta, getattr(st.wrapped, "comm_backend", None))
for model, parallel in CASES:
    a, b = out[(model, parallel, "0")], out[(model, parallel, "1")]
    assert "rccl" in str(b[2]).lower(), b[2]
    # a broken identity all-reduce (doubled or unreduced moments, a read racing
    # the collective) moves the loss by far more than this
    assert abs(a[0] - b[0]) < 1e-2 * max(1.0, abs(a[0])), (model, parallel, a[0], b[0])
    # whole-update cosine: MIOpen's weight gradients are not bit-deterministic
    # (profiles/README.md finding 4), so single small tensors (a BN bias) can drift
    # between two identical steps; an identity "average" must still keep the update
    # (0.988-0.991 measured between two identical resnet18 steps at batch 8);
    # the norm ratio catches a scaled "average" (sum instead of mean: 2x at ws 2)
    ua, ub = torch.cat([x.flatten() for x in a[1]]), torch.cat([y.flatten() for y in b[1]])
    cos = torch.nn.functional.cosine_similarity(ua, ub, dim=0).item()
    nrm = (ub.norm() / ua.norm()).item()
    # ResNet-50 at batch 8 / 64 px (2x2 maps in layer 4, batch-statistics BN) is
    # far more chaotic: 0.89 measured; a corrupted or racing identity all-reduce
    # at world size 1 gives garbage (cosine near 0) or NaN, not 0.8
    assert cos > (0.97 if model == "resnet18" else 0.8) and abs(nrm - 1) < 0.05, (model, parallel, cos, nrm)
    print(model, parallel, "ok", a[0], b[0], b[2], cos, nrm)
from distributed_model_parallel_amd.comm.rccl import default_communicator
comm = default_communicator(env.device)
t = torch.arange(10, dtype=torch.float64, device=env.device)
comm.all_reduce(t, "sum", on_current_stream=True)   # SyncBN's path
u = torch.arange(10, dtype=torch.float32, device=env.device)
comm.all_reduce(u, "avg")
comm.wait()
torch.cuda.synchronize()
assert torch.equal(t.cpu(), torch.arange(10, dtype=torch.float64)) and torch.equal(u.cpu(), torch.arange(10.0))
print("rccl on-current-stream ok")
destroy_distributed()
'''


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ddp_and_syncbn_rccl_backend_world1():
    env = dict(os.environ, ROOT=ROOT, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True,
                       timeout=900)
    if r.returncode != 0:
        print(r.stdout[-3000:])
        print(r.stderr[-6000:])
    assert r.returncode == 0, "subprocess failed (output above)"
    assert "resnet18 ddp ok" in r.stdout and "resnet18 syncbn ok" in r.stdout and "resnet50 syncbn ok" in r.stdout
    assert "rccl on-current-stream ok" in r.stdout


ORDER_SCRIPT = r'''
import os, sys, torch
import torch.nn.functional as F
sys.path.insert(0, os.environ["ROOT"])
from distributed_model_parallel_amd import _native
from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.ops.optim import FlatSGD, MasterSGD
from distributed_model_parallel_amd.parallel.data_parallel import DataParallel
from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
from distributed_model_parallel_amd.utils.env import init_distributed, destroy_distributed
from distributed_model_parallel_amd.utils.precision import cast_model
env = init_distributed()
dev = env.device
C = _native.require("test")
g = torch.Generator().manual_seed(3)
x = torch.randn(8, 3, 64, 64, generator=g).to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), generator=g).to(dev)

def model():
    torch.manual_seed(0)
    m = build_model("resnet18").to(dev).to(memory_format=torch.channels_last)
    cast_model(m, torch.bfloat16)
    return m

def masters_ddp(m, ddp, opt):
    opt._ensure_state()
    flats = [st.get("master", st["param"]).float() for st in opt._flat_state]
    return [flats[gi].narrow(0, off, p.numel()).clone() for p, (gi, off) in zip(ddp._params, ddp.param_layout())]

def masters_sgd(opt):
    out = {}
    for st in opt._groups:
        for p, off in zip(st["params"], st["offs"]):
            out[id(p)] = st.get("master", st["param"]).float().narrow(0, off, p.numel()).clone()
    return out

def ddp_step(backend=None):
    m = model()
    ddp = DistributedDataParallel(m, flat_parameters=True)
    if backend is not None:
        ddp.reducer.set_backend(backend(ddp))
    opt = FlatSGD(ddp, lr=1.0, momentum=0.0, weight_decay=0.0)
    w0 = masters_ddp(m, ddp, opt)
    F.cross_entropy(ddp(x).float(), y).backward()
    opt.step()
    torch.cuda.synchronize()
    return [a - b for a, b in zip(masters_ddp(m, ddp, opt), w0)]

# 1) ordering: the comm stream sleeps ~tens of ms, then doubles the averaged
#    gradient; FlatSGD on the compute stream must see the doubled value.
def rel_errs(xs, ys):
    return sorted(((a - b).norm() / (b.norm() + 1e-12)).item() for a, b in zip(xs, ys) if b.norm() > 0)

# one throwaway step first: MIOpen's find mode may pick a different algorithm
# on a shape's first use than on later ones, and a random-init ResNet-18 at
# batch 8 amplifies that rounding difference to ~10 % of the update (measured:
# 0.085 median once in a full-suite run, 6e-6 once warmed)
ddp_step()
base = ddp_step()
slow = ddp_step(lambda d: C.RcclReduceBackend(d.comm.native, 2.0, 200_000_000))
# MIOpen's weight gradients are not bit-deterministic (profiles/README.md finding 4),
# so compare per parameter with a noise allowance; a missing event makes the
# optimizer see the UNdoubled gradient: relative error 0.5 on every parameter it
# hits.  Measured noise between two correct steps: median 6e-6 warmed, but
# 0.085 (max 0.10) in two full-suite runs -- the random-init ResNet-18 at batch
# 8 amplifies one nondeterministic sum chaotically -- so the signature checked
# is "no parameter near 0.5", with the median well under it
errs = rel_errs(slow, [2 * b for b in base])
assert errs[len(errs) // 2] < 0.2 and errs[-1] < 0.35, ("optimizer read the gradient before the comm stream finished", errs[len(errs) // 2], errs[-1])
print("ordering ok", errs[len(errs) // 2], errs[-1])

# 2) precision parity: one bf16 DP step (device_ids=[0]) and one bf16 DDP step
#    produce the same fp32 master update.
m = model()
opt = MasterSGD(m.parameters(), lr=1.0)
dp = DataParallel(m, device_ids=[0])
w0 = masters_sgd(opt)
F.cross_entropy(dp(x).float(), y).backward()
opt.step()
torch.cuda.synchronize()
w1 = masters_sgd(opt)
dps = [w1[id(p)] - w0[id(p)] for p in m.parameters()]
errs = rel_errs(dps, base)
pn = [n for n, _ in m.named_parameters()]
print("dp-ddp worst", sorted(((((a - b).norm() / (b.norm() + 1e-12)).item(), n) for n, a, b in zip(pn, dps, base)), reverse=True)[:6])
print("ddp-ddp noise", sorted(((((a - 2 * b).norm() / (2 * b.norm() + 1e-12)).item(), n) for n, a, b in zip(pn, slow, base)), reverse=True)[:6])
# DP and DDP run different (equally exact) backward code paths -- e.g. DDP's
# fused BN-backward epilogues vs DP replicas -- whose bf16 rounding differences
# a random-init ResNet amplifies chaotically (profiles/README.md finding 4:
# per-parameter cosines fall to ~0.2 at tiny batches), so parity is judged on
# the whole update: a bf16-only (no fp32 master) step, a missing weight-decay /
# momentum term or a stale gradient moves it far more than this
cos = F.cosine_similarity(torch.cat([a.flatten() for a in dps]), torch.cat([b.flatten() for b in base]), dim=0).item()
nrm = (torch.cat([a.flatten() for a in dps]).norm() / torch.cat([b.flatten() for b in base]).norm()).item()
assert cos > 0.98 and abs(nrm - 1) < 0.05 and errs[len(errs) // 2] < 0.15, ("DP and DDP master updates differ", cos, nrm, errs[len(errs) // 2])
print("dp-ddp parity ok", cos, nrm, errs[len(errs) // 2], errs[-1])
destroy_distributed()
'''


def test_reducer_stream_ordering_and_dp_ddp_precision_parity():
    env = dict(os.environ, ROOT=ROOT, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", ORDER_SCRIPT], env=env, capture_output=True, text=True,
                       timeout=600)
    print(r.stdout[-3000:])
    if r.returncode != 0:
        print(r.stderr[-6000:])
    assert r.returncode == 0, "subprocess failed (output above)"
    assert "ordering ok" in r.stdout and "dp-ddp parity ok" in r.stdout
