#!/usr/bin/env python3
"""Stock-PyTorch comparison point for bench.py (same model / batch / dtype).

A plain torchvision-equivalent ResNet-50 built ONLY from stock modules --
nn.Conv2d (MIOpen), nn.BatchNorm2d, nn.ReLU, nn.MaxPool2d,
nn.AdaptiveAvgPool2d, nn.Linear -- none of this repo's ops; channels-last;
bf16 weights (or fp32 weights + bf16 autocast); torch DistributedDataParallel;
torch.optim.SGD(foreach).  MIOpen find is ON by default (cudnn.benchmark=1)
and seeded from the same committed find db the bench uses, so the stock convs
get their tuned solutions.  Used only to measure what the native path buys;
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
from distributed_model_parallel_amd.utils import miopen_db  # noqa: E402


class StockBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        return self.relu(self.bn3(self.conv3(out)) + idt)


class StockResNet50(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        layers, cin = [], 64
        for planes, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            ds = None
            if stride != 1 or cin != planes * 4:
                ds = nn.Sequential(nn.Conv2d(cin, planes * 4, 1, stride, bias=False),
                                   nn.BatchNorm2d(planes * 4))
            blocks = [StockBottleneck(cin, planes, stride, ds)]
            cin = planes * 4
            blocks += [StockBottleneck(cin, planes) for _ in range(1, n)]
            layers.append(nn.Sequential(*blocks))
        self.layers = nn.Sequential(*layers)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.avgpool(self.layers(x)).flatten(1)
        return self.fc(x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--mode", default="bf16", choices=["bf16", "amp"])
    ap.add_argument("--benchmark", type=int, default=1, help="MIOpen find (cudnn.benchmark)")
    ap.add_argument("--miopen-db", default="use", choices=["use", "off"])
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dist.init_process_group("nccl", rank=int(os.environ.get("RANK", 0)),
                            world_size=int(os.environ.get("WORLD_SIZE", 1)))
    lr = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(lr)
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    miopen_db.seed(a.miopen_db)
    m = StockResNet50().cuda().to(memory_format=torch.channels_last)
    assert sum(p.numel() for p in m.parameters()) == 25_557_032
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
    import threading
    done = threading.Event()

    def heartbeat():  # MIOpen find over every stock conv can take minutes in step 0
        while not done.wait(30):
            print(f"  ... still warming up at {time.time() - t:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()
    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()  # MIOpen find runs in the first steps: report progress
        print(f"warmup step {i} done at {time.time()-t:.1f}s", file=sys.stderr, flush=True)
    done.set()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ws = dist.get_world_size()
    print(json.dumps({"baseline": "stock-pytorch (nn.Conv2d/BatchNorm2d/MaxPool2d only)", "mode": a.mode,
                      "benchmark": a.benchmark, "batch": a.batch_size,
                      "images_per_sec": a.batch_size * ws * a.steps / el,
                      "ms_per_step": 1000 * el / a.steps, "loss": float(loss)}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
