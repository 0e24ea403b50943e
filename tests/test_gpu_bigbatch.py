"""Large-batch guard for the headline configuration (ResNet-50 bf16 channels-last,
per-GPU batch 2048): activations of 1.6 G elements / 3.3 GB per tensor, so any
32-bit byte offset in a native kernel would wrap there and nowhere in the small
numerics tests.

A batch made of the same 1024 images twice has exactly the training-mode BN
statistics of the 1024 images alone and the same mean cross-entropy, and its two
halves must produce the same activations and input gradients; a wrapped offset
breaks that symmetry.  (The parameter gradients are not compared exactly: a
random-init ResNet-50 amplifies reduction-order differences chaotically,
profiles/README.md finding 4.)  The comparison runs in one subprocess (the model at this
size needs ~80 GB; nothing else is resident)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import os, sys, torch
import torch.nn.functional as F
sys.path.insert(0, os.environ["ROOT"])
from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.utils.precision import cast_model
from distributed_model_parallel_amd.ops import batchnorm as bn
from distributed_model_parallel_amd.utils import miopen_db
torch.backends.cudnn.benchmark = True   # the bench's MIOpen setup: find, seeded db,
miopen_db.seed("use")                   # naive reference solvers excluded
dev = torch.device("cuda:0")
torch.manual_seed(0)
m = build_model("resnet50").to(dev).to(memory_format=torch.channels_last)
cast_model(m, torch.bfloat16)
g = torch.Generator().manual_seed(5)
x = torch.randn(1024, 3, 224, 224, generator=g).to(dev, torch.bfloat16)
y = torch.randint(0, 1000, (1024,), generator=g).to(dev)

def run(xb, yb):
    for p in m.parameters():
        p.grad = None
    loss = F.cross_entropy(m(xb.contiguous(memory_format=torch.channels_last)).float(), yb)
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()])

names = [n for n, _ in m.named_parameters()]
l1, g1 = run(x, y)
print("1024 done", file=sys.stderr, flush=True)
# the duplicated batch: every per-sample path of the second half runs at
# offsets past 2^31 bytes in the big activations (layer 1: 2048 x 56 x 56 x 256
# bf16 = 3.3 GB), the first half below; with shared BN statistics the two halves
# must agree -- forward activations and input gradients -- up to reduction order
acts = []
hooks = [mod.register_forward_hook(lambda _m, _i, o: acts.append(o.detach()))
         for mod in m.modules() if type(mod).__name__ in ("Bottleneck", "BasicBlock")]
xx = torch.cat([x, x]).contiguous(memory_format=torch.channels_last).requires_grad_(True)
for p in m.parameters():
    p.grad = None
loss2 = F.cross_entropy(m(xx).float(), torch.cat([y, y]))
loss2.backward()
torch.cuda.synchronize()
for h in hooks:
    h.remove()
l2 = loss2.item()
g2 = torch.cat([p.grad.float().flatten() for p in m.parameters()])
worst_act = max(((a[:1024].float() - a[1024:].float()).norm() / a[:1024].float().norm()).item() for a in acts)
d = xx.grad.float()
dx_rel = ((d[:1024] - d[1024:]).norm() / d[:1024].norm()).item()
cos = F.cosine_similarity(g1, g2, dim=0).item()
print(f"loss 1024 {l1:.5f} 2048-dup {l2:.5f}; {len(acts)} block outputs, worst half-vs-half rel {worst_act:.2e}; "
      f"input-grad half-vs-half rel {dx_rel:.2e}; param-grad cos vs 1024 {cos:.4f} (chaotic, not asserted); "
      f"bn {bn.stats()}", flush=True)
assert abs(l1 - l2) < 2e-3 * abs(l1), (l1, l2)
assert bool(torch.isfinite(g2).all()) and bool(torch.isfinite(d).all())
assert len(acts) == 16 and worst_act < 1e-2, worst_act
assert dx_rel < 2e-2, dx_rel
print("bigbatch ok")
'''


def test_resnet50_batch2048_matches_duplicated_1024():
    env = dict(os.environ, ROOT=ROOT)
    # output streams through (a long silent child would look hung to the runner)
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, stdout=subprocess.PIPE, text=True,
                       timeout=600)
    print(r.stdout[-3000:])
    assert r.returncode == 0 and "bigbatch ok" in r.stdout
