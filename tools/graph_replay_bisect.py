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
        if step == 0 or not os.environ.get("SAMEX"):
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
        if os.environ.get("VERBOSE"):
            for (pn, pa), pg in zip(A.named_parameters(), Gm.parameters()):
                if pa.grad is not None and pg.grad is not None:
                    d = (pa.grad.float() - pg.grad.float()).abs().max().item()
                    if not d < 1e-2 * max(pa.grad.float().abs().max().item(), 1e-6):
                        line.append(f"   {pn} {tuple(pa.shape)} max|dA| {pa.grad.float().abs().max().item():.3g} "
                                    f"max|dG| {pg.grad.float().abs().max().item():.3g}")
        for o in opts:
            if not os.environ.get("NOUPDATE"):
                o.step()
            # ZERO_GRADS=1: keep zeroed .grad tensors (AccumulateGrad adds into them
            # instead of stealing the graph's static gradient buffers)
            o.zero_grad(set_to_none=not os.environ.get("ZERO_GRADS"))
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
    from distributed_model_parallel_amd.models.resnet import BasicBlock
    from distributed_model_parallel_amd.ops.batchnorm import BatchNormAct2d

    def cbr(c, relu=True):
        return [torch.nn.Conv2d(c, c, 3, padding=1, bias=False), BatchNormAct2d(c, act="relu" if relu else None)]

    def mk(mods):
        m = torch.nn.Sequential(*mods).cuda().to(memory_format=torch.channels_last)
        cast_model(m, torch.bfloat16)
        return m
    pieces += [("cbr512", mk(cbr(512)), (n, 512, 2, 2)), ("cbr512x2", mk(cbr(512) + cbr(512)), (n, 512, 2, 2)),
               ("cbr512x3", mk(cbr(512) + cbr(512) + cbr(512)), (n, 512, 2, 2)),
               ("cb512x2_norelu", mk(cbr(512, False) + cbr(512, False)), (n, 512, 2, 2)),
               ("block512x2", mk([BasicBlock(512, 512), BasicBlock(512, 512)]), (n, 512, 2, 2)),
               ("cbr256x2_4x4", mk(cbr(256) + cbr(256)), (n, 256, 4, 4)),
               ("cbr64x2_16x16", mk(cbr(64) + cbr(64)), (n, 64, 16, 16)),
               ("bnrelu512", mk([BatchNormAct2d(512, act="relu")]), (n, 512, 2, 2)),
               ("bn512", mk([BatchNormAct2d(512)]), (n, 512, 2, 2)),
               ("conv_bn_stockrelu", mk([torch.nn.Conv2d(512, 512, 3, padding=1, bias=False), BatchNormAct2d(512),
                                         torch.nn.ReLU()]), (n, 512, 2, 2)),
               ("conv_stockrelu", mk([torch.nn.Conv2d(512, 512, 3, padding=1, bias=False), torch.nn.ReLU()]),
                (n, 512, 2, 2)),
               ("conv_only", mk([torch.nn.Conv2d(512, 512, 3, padding=1, bias=False)]), (n, 512, 2, 2)),
               ("conv1x1_bnrelu", mk([torch.nn.Conv2d(512, 512, 1, bias=False), BatchNormAct2d(512, act="relu")]),
                (n, 512, 2, 2)),
               ("cbr512_16x16", mk(cbr(512)), (n, 512, 16, 16))]
    only = os.environ.get("ONLY")
    for name, mod, shp in pieces:
        if only and name not in only.split(","):
            continue
        try:
            check(name, copy.deepcopy(mod), shp)
        except Exception as e:  # report and go on to the next piece
            print(f"== {name}: {type(e).__name__}: {e}", flush=True)


if __name__ == "__main__":
    if os.environ.get("REFMODE"):  # every op on its stock-PyTorch path
        from distributed_model_parallel_amd import _native
        with _native.reference_mode():
            main()
    else:
        main()
