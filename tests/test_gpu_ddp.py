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
for parallel in ("ddp", "syncbn"):
    for forced in ("0", "1"):
        os.environ["DMP_DDP_SINGLE_RANK_COMM"] = forced
        cfg = StepConfig(model="resnet18", batch_size=8, image_size=64, parallel=parallel)
        st = build_train_state(cfg, env.device)
        before = [p.detach().float().clone() for p in st.model.parameters()]
        loss = st.step()          # one step: the update carries the (averaged) gradient
        torch.cuda.synchronize()
        delta = [p.detach().float() - b for p, b in zip(st.model.parameters(), before)]
        out[(parallel, forced)] = (loss.item(), delta, getattr(st.wrapped, "comm_backend", None))
for parallel in ("ddp", "syncbn"):
    a, b = out[(parallel, "0")], out[(parallel, "1")]
    assert "rccl" in str(b[2]).lower(), b[2]
    assert abs(a[0] - b[0]) < 1e-3 * max(1.0, abs(a[0])), (parallel, a[0], b[0])
    cos = min(torch.nn.functional.cosine_similarity(x.flatten(), y.flatten(), dim=0).item()
              for x, y in zip(a[1], b[1]) if y.norm() > 0)
    assert cos > 0.98, (parallel, cos)
    print(parallel, "ok", a[0], b[0], b[2], cos)
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
    assert "ddp ok" in r.stdout and "syncbn ok" in r.stdout
    assert "rccl on-current-stream ok" in r.stdout
