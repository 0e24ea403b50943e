"""Whole-step hipGraph capture (train/graphed.py): after eager warm-up, replaying
the captured DDP training step (forward, backward with the C++ reducer, fused
flat SGD) must track the eager trajectory.  Subprocess: the process group is
process-global."""
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
model = os.environ["MODEL"]
res = {}
for graph in (False, True):
    cfg = StepConfig(model=model, batch_size=16, image_size=int(os.environ["IMG"]), graph=graph,
                     lr=0.01)
    st = build_train_state(cfg, env.device)
    losses = [float(st.step()) for _ in range(6)]
    torch.cuda.synchronize()
    res[graph] = losses
    print("graph" if graph else "eager", losses)
e, g = res[False], res[True]
# MIOpen's weight gradients are non-deterministic and the 16-sample loss falls
# fast (7 -> 0.3 in six steps), so the trajectories drift apart: tight for the
# first two steps, looser once the drift compounds
for i, (a, b) in enumerate(zip(e, g)):
    tol = 2e-2 if i < 2 else 1.5e-1
    assert abs(a - b) <= tol * max(1.0, abs(a)), (e, g)
assert g[-1] != g[3], "replays did not advance the training state"
destroy_distributed()
'''


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("model,img", [("resnet18", 64), ("mobilenetv2", 32)])
def test_graphed_step_tracks_eager(model, img):
    env = dict(os.environ, ROOT=ROOT, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MODEL=model,
               IMG=str(img), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, "-c", SCRIPT], env=env, capture_output=True, text=True,
                       timeout=900)
    if r.returncode != 0:
        print(r.stdout[-3000:])
        print(r.stderr[-6000:])
    assert r.returncode == 0, "subprocess failed (output above)"
