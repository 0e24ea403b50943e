#!/usr/bin/env python3
"""Does a model captured with torch.cuda.make_graphed_callables replay the
same forward / backward as the eager model, step after step (new inputs and
SGD updates between replays)?  Prints, per step, the output difference and the
parameter gradients that differ (relative norm) or are non-finite.  Run it
under DMP_DISABLE=<feature> to bisect a route that is not replay-safe.

usage: python tools/graph_replay_check.py [--arch resnet18] [--size 64] [--batch 4] [--steps 3]
"""
import argparse
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="resnet18")
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lr", type=float, default=0.05)
    a = ap.parse_args()
    from distributed_model_parallel_amd.models import build_model
    from distributed_model_parallel_amd.ops.loss import cross_entropy
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(0)
    m_e = build_model(a.arch, num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_model(m_e, torch.bfloat16)
    m_g = copy.deepcopy(m_e)
    shape = (a.batch, 3, a.size, a.size)
    sx = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    saved = [b.detach().clone() for b in m_g.buffers()]
    g = torch.cuda.make_graphed_callables(m_g, (sx,))
    with torch.no_grad():
        for b, v in zip(m_g.buffers(), saved):
            b.copy_(v)
    opts = [torch.optim.SGD(m.parameters(), lr=a.lr) for m in (m_e, m_g)]
    print(f"DMP_DISABLE={os.environ.get('DMP_DISABLE', '')!r}")
    for step in range(a.steps):
        x = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        y = torch.arange(a.batch, device="cuda") % 10
        out_e = m_e(x)
        cross_entropy(out_e, y).backward()
        sx.copy_(x)
        out_g = g(sx)
        cross_entropy(out_g, y).backward()
        torch.cuda.synchronize()
        d = (out_e.float() - out_g.float()).abs().max().item()
        rows, bad = [], []
        for (n, pe), pg in zip(m_e.named_parameters(), m_g.parameters()):
            ge = pe.grad.float()
            gg = pg.grad.float() if pg.grad is not None else torch.zeros_like(ge)
            if not torch.isfinite(gg).all():
                bad.append(n)
                continue
            rows.append(((gg - ge).norm().item() / max(ge.norm().item(), 1e-12), n))
        rows.sort(reverse=True)
        print(f"step {step}: output max diff {d:.4g}; non-finite grads {len(bad)} {bad[:6]}; "
              f"worst rel {[f'{r:.3g} {n}' for r, n in rows[:3]]}; median rel {rows[len(rows) // 2][0]:.3g}",
              flush=True)
        for opt in opts:
            opt.step()
            opt.zero_grad()


if __name__ == "__main__":
    main()
