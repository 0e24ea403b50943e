#!/usr/bin/env python3
"""Diagnose whole-step hipGraph capture: prints each phase (warm-up, capture,
replay) with faulthandler on, for --parallel none|ddp and a chosen model."""
import argparse
import faulthandler
import os
import sys

import torch

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.env import init_distributed  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet18")
ap.add_argument("--img", type=int, default=64)
ap.add_argument("--parallel", default="ddp")
ap.add_argument("--bs", type=int, default=16)
a = ap.parse_args()
env = init_distributed()
cfg = StepConfig(model=a.model, batch_size=a.bs, image_size=a.img, parallel=a.parallel, lr=0.01)
side = torch.cuda.Stream()
with torch.cuda.stream(side):  # build on the capture stream (see train/step.py)
    st = build_train_state(cfg, env.device)
step = st.step
for i in range(3):
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        loss = step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print(f"warmup {i} loss {float(loss):.4f}", flush=True)
g = torch.cuda.CUDAGraph()
print("capture begin", flush=True)
with torch.cuda.graph(g, stream=side):
    out = step()
print("capture end", flush=True)
torch.cuda.synchronize()
for i in range(3):
    g.replay()
    torch.cuda.synchronize()
    print(f"replay {i} loss {float(out):.4f}", flush=True)
print("ok", flush=True)
