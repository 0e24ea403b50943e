#!/usr/bin/env python3
"""Whole-model train-mode gradient parity of the native bf16 ResNet-50 step
against stock PyTorch fp32 on the same weights and input.

Prints, per configuration (batch, image size, residual-branch gamma):
  native bf16 vs stock fp32, stock bf16 vs stock fp32, native vs native
  (a second native run: atomic-order noise) and stock fp32 vs stock fp32
  with the input perturbed by one fp32 ulp -- per-parameter gradient cosine
  (median / 5th percentile / min, worst parameter) and the loss difference.

usage: python tools/parity_probe.py [--batch 32 64] [--size 224] [--gamma 0.25 1.0]
"""
from __future__ import annotations

import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.models import build_model  # noqa: E402
from distributed_model_parallel_amd.ops.loss import cross_entropy  # noqa: E402
from distributed_model_parallel_amd.utils.precision import cast_model  # noqa: E402


def build(gamma: float, ncls: int, seed: int = 0):
    torch.manual_seed(seed)
    m = build_model("resnet50", num_classes=ncls)
    with torch.no_grad():
        for mod in m.modules():
            if hasattr(mod, "bn3"):
                mod.bn3.weight.mul_(gamma)
    return m


def grads_native(m0, x, y, tn_all: bool = True):
    from distributed_model_parallel_amd.ops import conv1x1
    m = copy.deepcopy(m0).cuda().to(memory_format=torch.channels_last)
    cast_model(m, torch.bfloat16)
    old = conv1x1._TN_XL_MIN_ROWS
    if tn_all:
        conv1x1._TN_XL_MIN_ROWS = 0  # the bench's batch-2048 ping-pong TN route at this batch too
    try:
        loss = cross_entropy(m(x.bfloat16().contiguous(memory_format=torch.channels_last)), y)
        loss.backward()
    finally:
        conv1x1._TN_XL_MIN_ROWS = old
    return float(loss.detach()), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def grads_stock(m0, x, y, dtype=torch.float32):
    m = copy.deepcopy(m0).cuda().to(memory_format=torch.channels_last).to(dtype)
    with _native.reference_mode():
        loss = torch.nn.functional.cross_entropy(m(x.to(dtype).contiguous(memory_format=torch.channels_last)).float(), y)
        loss.backward()
    return float(loss), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def compare(a, b):
    cs = []
    for n in a:
        ga, gb = a[n].flatten(), b[n].flatten()
        den = (ga.norm() * gb.norm()).item()
        cs.append(((ga @ gb).item() / den if den > 0 else 1.0, n))
    cs.sort()
    vals = torch.tensor([c for c, _ in cs])
    conv = torch.tensor([c for c, n in cs if n.endswith("weight") and a[n].dim() == 4])
    fa = torch.cat([a[n].flatten() for n in a])
    fb = torch.cat([b[n].flatten() for n in a])
    whole = ((fa @ fb) / (fa.norm() * fb.norm()).clamp_min(1e-30)).item()
    return {"median": vals.median().item(), "p05": vals.quantile(0.05).item(), "min": cs[0][0],
            "worst": cs[0][1], "conv_median": conv.median().item(), "conv_min": conv.min().item(),
            "whole": whole}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--gamma", type=float, nargs="+", default=[0.25, 1.0])
    ap.add_argument("--classes", type=int, default=100)
    a = ap.parse_args()
    for gamma in a.gamma:
        m0 = build(gamma, a.classes)
        for batch in a.batch:
            g = torch.Generator().manual_seed(7)
            x = torch.randn(batch, 3, a.size, a.size, generator=g).bfloat16().float().cuda()
            y = torch.randint(0, a.classes, (batch,), generator=g).cuda()
            l32, g32 = grads_stock(m0, x, y)
            xp = x * (1 + 2 ** -23)
            l32p, g32p = grads_stock(m0, xp, y)
            l16, g16 = grads_stock(m0, x, y, torch.bfloat16)
            ln, gn = grads_native(m0, x, y)
            ln2, gn2 = grads_native(m0, x, y)
            rows = [("native bf16 vs stock fp32", compare(gn, g32), ln, l32),
                    ("stock bf16 vs stock fp32", compare(g16, g32), l16, l32),
                    ("native vs native (run 2)", compare(gn, gn2), ln, ln2),
                    ("stock fp32 vs fp32, input +1 ulp", compare(g32p, g32), l32p, l32)]
            print(f"\n## gamma {gamma}, batch {batch}, {a.size} px\n")
            print("| pair | median cos | p05 | min | worst parameter | conv median | conv min | whole-model cos "
                  "| loss a | loss b | rel |")
            print("|---|---|---|---|---|---|---|---|---|---|---|")
            for name, c, la, lb in rows:
                print(f"| {name} | {c['median']:.5f} | {c['p05']:.5f} | {c['min']:.5f} | {c['worst']} | "
                      f"{c['conv_median']:.5f} | {c['conv_min']:.5f} | {c['whole']:.5f} | "
                      f"{la:.5f} | {lb:.5f} | {abs(la - lb) / abs(lb):.2e} |", flush=True)
            torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
