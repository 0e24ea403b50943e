#!/usr/bin/env python3
"""Diagnostic: DataParallel(graphs=True) vs the eager replica path on one
step -- per-parameter relative gradient error, worst first, plus the output
error.  usage: python tools/dp_graph_diag.py [--arch resnet18] [--replicas 4]"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--lr", type=float, default=0.05)
    a = ap.parse_args()
    from distributed_model_parallel_amd.models import build_model
    from distributed_model_parallel_amd.ops.loss import cross_entropy
    from distributed_model_parallel_amd.parallel.data_parallel import DataParallel
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(0)
    base = build_model(a.arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_model(base, torch.bfloat16)
    m_e, m_g, m_s = base, copy.deepcopy(base), copy.deepcopy(base)
    devs = [0] * a.replicas
    dp_e = DataParallel(m_e, device_ids=devs)
    dp_g = DataParallel(m_g, device_ids=devs, graphs=True)
    opts = [torch.optim.SGD(m.parameters(), lr=a.lr) for m in (m_e, m_g, m_s)]
    for step in range(a.steps):
        x = torch.randn(a.batch, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.arange(a.batch, device="cuda") % 10
        outs, losses = {}, {}
        # reference: one module, the replicas' chunks one after another (per-chunk
        # BN statistics, as DataParallel), outputs concatenated before the loss
        for name, fn in (("eager", dp_e), ("graphed", dp_g),
                         ("single", lambda v: torch.cat([m_s(c) for c in v.chunk(a.replicas)]))):
            out = fn(x)
            loss = cross_entropy(out, y)
            loss.backward()
            outs[name], losses[name] = out.float(), loss.item()
        print(f"=== step {step}: loss", {k: round(v, 4) for k, v in losses.items()})
        for k in ("eager", "graphed"):
            print(f"output max abs diff {k} vs single", (outs[k] - outs["single"]).abs().max().item())
        for k, mod in (("eager", m_e), ("graphed", m_g)):
            rows = []
            bad = 0
            for (n, ps), pk in zip(m_s.named_parameters(), mod.parameters()):
                gs = ps.grad.float()
                gk = pk.grad.float() if pk.grad is not None else torch.zeros_like(gs)
                bad += int(not torch.isfinite(gk).all())
                rel = ((gk - gs).norm() / gs.norm().clamp_min(1e-12)).item()
                rows.append((rel, n, tuple(ps.shape), gs.norm().item(), gk.norm().item()))
            rows.sort(reverse=True)
            print(f"--- {k} vs single: {bad} non-finite parameter gradients; worst:")
            for rel, n, shp, ns, nk in rows[:8]:
                print(f"{rel:9.4f}  {n:40s} {str(shp):22s} |single| {ns:.4e} |{k}| {nk:.4e}")
            print("median rel", sorted(r[0] for r in rows)[len(rows) // 2])
        for opt in opts:
            opt.step()
            opt.zero_grad()


if __name__ == "__main__":
    main()
