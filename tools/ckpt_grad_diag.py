#!/usr/bin/env python3
"""Gradient agreement of one ResNet-50 training step at a tiny batch between
the fused native path, the checkpointed (unfused) native path and a stock fp32
PyTorch oracle of the same weights (_native.reference_mode), per top-level
stage: is a low fused-vs-checkpointed cosine rounding chaos (both bf16 paths
equally far from fp32) or one path being wrong (that path far, the other near)?

usage: python tools/ckpt_grad_diag.py [--batch 8] [--size 64] [--seeds 3]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.models import build_model  # noqa: E402
from distributed_model_parallel_amd.ops.loss import cross_entropy  # noqa: E402
from distributed_model_parallel_amd.utils.checkpointing import enable_activation_checkpointing  # noqa: E402
from distributed_model_parallel_amd.utils.precision import cast_model  # noqa: E402


def stage_grads(m):
    out = {}
    for n, p in m.named_parameters():
        k = n.split(".")[0]
        out.setdefault(k, []).append(p.grad.float().flatten())
    return {k: torch.cat(v) for k, v in out.items()}


def cos(a, b):
    return torch.nn.functional.cosine_similarity(a, b, dim=0).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--seeds", type=int, default=3)
    args = ap.parse_args()
    CL = torch.channels_last
    for seed in range(args.seeds):
        torch.manual_seed(seed)
        base = build_model("resnet50", num_classes=10).cuda().to(memory_format=CL)
        ref = copy.deepcopy(base)  # fp32 oracle, same weights
        cast_model(base, torch.bfloat16)
        fused, ckpt = copy.deepcopy(base), copy.deepcopy(base)
        enable_activation_checkpointing(ckpt, 4)
        x = torch.randn(args.batch, 3, args.size, args.size, device="cuda").contiguous(memory_format=CL)
        y = torch.arange(args.batch, device="cuda") % 10
        cross_entropy(fused(x.bfloat16()), y).backward()
        cross_entropy(ckpt(x.bfloat16()), y).backward()
        with _native.reference_mode():
            cross_entropy(ref(x), y).backward()
        gf, gc, gr = stage_grads(fused), stage_grads(ckpt), stage_grads(ref)
        allf, allc, allr = (torch.cat(list(g.values())) for g in (gf, gc, gr))
        print(f"seed {seed}: whole model  fused~fp32 {cos(allf, allr):.4f}  ckpt~fp32 {cos(allc, allr):.4f}  "
              f"fused~ckpt {cos(allf, allc):.4f}", flush=True)
        for k in gr:
            print(f"    {k:8s} fused~fp32 {cos(gf[k], gr[k]):.4f}  ckpt~fp32 {cos(gc[k], gr[k]):.4f}  "
                  f"fused~ckpt {cos(gf[k], gc[k]):.4f}  |g| fp32 {gr[k].norm().item():.3e}", flush=True)
        del base, ref, fused, ckpt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
