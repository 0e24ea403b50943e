#!/usr/bin/env python3
"""Bisect which module of ResNet-18 (64 px, batch 4) is not replay-safe under
torch.cuda.make_graphed_callables, and whether two EAGER copies of the same
module agree at all (first-call algorithm searches, reads of uninitialised
memory).  For every piece: an eager copy A, an eager copy B and a graphed copy
G, fed the same inputs and output gradients for 4 steps with SGD updates in
between; prints the max output difference and the relative parameter-gradient
difference of B and G against A, and any non-finite gradients."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(ma, mb):
    num = den = 0.0
    bad = 0
    for a, b in zip(ma.parameters(), mb.parameters()):
        if a.grad is None or b.grad is None:
            continue
        if not torch.isfinite(b.grad).all():
            bad += 1
            continue
        num += (a.grad.float() - b.grad.float()).pow(2).sum().item()
        den += a.grad.float().pow(2).sum().item()
    return (num / max(den, 1e-30)) ** 0.5, bad


def check(name, mod, in_shape, steps=4, lr=0.05):
    torch.manual_seed(1)
    A = mod
    B = copy.deepcopy(A)
    Gm = copy.deepcopy(A)
    sx = torch.randn(in_shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    saved = [b.detach().clone() for b in Gm.buffers()]
    G = torch.cuda.make_graphed_callables(Gm, (sx,))
    with torch.no_grad():
        for b, v in zip(Gm.buffers(), saved):
            b.copy_(v)
    opts = [torch.optim.SGD(m.parameters(), lr=lr) for m in (A, B, Gm)]
    line = []
    for step in range(steps):
        x = torch.randn(in_shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        outs = []
        go = None
        for fn, m in ((A, A), (B, B), (G, Gm)):
            if fn is G:
                sx.copy_(x)
                o = G(sx)
            else:
                o = fn(x)
            if go is None:
                go = torch.randn_like(o)
            o.backward(go)
            outs.append(o.float())
        torch.cuda.synchronize()
        rb, bb = rel(A, B)
        rg, bg = rel(A, Gm)
        line.append(f"s{step}: out B {(outs[1] - outs[0]).abs().max().item():.3g} G {(outs[2] - outs[0]).abs().max().item():.3g}"
                    f" | grad B {rb:.3g} G {rg:.3g}" + (f" NONFINITE G {bg}" if bg else "") + (f" NONFINITE B {bb}" if bb else ""))
        for o in opts:
            o.step()
            o.zero_grad()
    print(f"== {name}\n   " + "\n   ".join(line), flush=True)


def main():
    from distributed_model_parallel_amd.models import build_model
    from distributed_model_parallel_amd.utils.precision import cast_model
    torch.manual_seed(0)
    net = build_model("resnet18", num_classes=10).cuda().to(memory_format=torch.channels_last)
    cast_model(net, torch.bfloat16)
    n = 4
    pieces = [("layer4", net.layer4, (n, 256, 4, 4)), ("layer4[0]", net.layer4[0], (n, 256, 4, 4)),
              ("layer4[1]", net.layer4[1], (n, 512, 2, 2)), ("layer3", net.layer3, (n, 128, 8, 8)),
              ("layer3[1]", net.layer3[1], (n, 256, 4, 4)), ("layer3[1].conv2", net.layer3[1].conv2, (n, 256, 4, 4)),
              ("layer1", net.layer1, (n, 64, 16, 16)), ("layer2", net.layer2, (n, 64, 16, 16)),
              ("whole", net, (n, 3, 64, 64))]
    only = os.environ.get("ONLY")
    for name, mod, shp in pieces:
        if only and name not in only.split(","):
            continue
        try:
            check(name, copy.deepcopy(mod), shp)
        except Exception as e:  # report and go on to the next piece
            print(f"== {name}: {type(e).__name__}: {e}", flush=True)


if __name__ == "__main__":
    main()
