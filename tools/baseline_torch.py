#!/usr/bin/env python3
"""Stock-PyTorch comparison point for bench.py (same model / batch / dtype):
torchvision-equivalent ResNet-50 with nn.BatchNorm2d (MIOpen), channels-last,
bf16 weights (or autocast), torch.nn.parallel.DistributedDataParallel and
torch.optim.SGD(foreach).  Used only to measure how much the native path buys;
NOT part of the framework."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.models import resnet  # noqa: E402


def plain_resnet50():
    """Our ResNet-50 with every fused BN swapped for nn.BatchNorm2d + explicit ReLU."""
    m = resnet.resnet50()

    class BNAct(nn.Module):
        def __init__(self, src):
            super().__init__()
            self.bn = nn.BatchNorm2d(src.num_features)
            self.relu = src.act == "relu"

        def forward(self, x, residual=None):
            y = self.bn(x)
            if residual is not None:
                y = y + residual
            return F.relu(y) if self.relu else y

    def swap(mod):
        for name, ch in mod.named_children():
            if isinstance(ch, nn.BatchNorm2d):
                setattr(mod, name, BNAct(ch))
            else:
                swap(ch)
    swap(m)
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--mode", default="bf16", choices=["bf16", "amp"])
    ap.add_argument("--benchmark", type=int, default=0)
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dist.init_process_group("nccl", rank=int(os.environ.get("RANK", 0)),
                            world_size=int(os.environ.get("WORLD_SIZE", 1)))
    lr = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(lr)
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    m = plain_resnet50().cuda().to(memory_format=torch.channels_last)
    dt = torch.bfloat16
    if a.mode == "bf16":
        m = m.to(dt)
    ddp = nn.parallel.DistributedDataParallel(m, device_ids=[lr], gradient_as_bucket_view=True)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, foreach=True)
    x = torch.randn(a.batch_size, 3, 224, 224, device="cuda", dtype=dt if a.mode == "bf16" else torch.float32)
    x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch_size,), device="cuda")

    def step():
        with torch.autocast("cuda", dtype=dt, enabled=a.mode == "amp"):
            out = ddp(x)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)
        return loss

    t = time.time()
    for i in range(a.warmup):
        step()
        if i == 0:
            torch.cuda.synchronize()
            print(f"first step {time.time()-t:.1f}s", file=sys.stderr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ws = dist.get_world_size()
    print(json.dumps({"baseline": "stock-pytorch", "mode": a.mode, "benchmark": a.benchmark,
                      "images_per_sec": a.batch_size * ws * a.steps / el,
                      "ms_per_step": 1000 * el / a.steps, "loss": float(loss)}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
