#!/usr/bin/env python3
"""How sensitive are a bf16 model's gradients to last-bit noise?  Compares
per-parameter gradient cosine between (a) igemm vs MIOpen 3x3 convs and
(b) MIOpen vs MIOpen with a 1-ulp perturbation of the input.  Diagnostic."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.models import build_model  # noqa: E402
from distributed_model_parallel_amd.ops import conv_igemm  # noqa: E402
from distributed_model_parallel_amd.utils.precision import cast_model  # noqa: E402


def grads(m, x, y):
    m.zero_grad(set_to_none=True)
    loss = F.cross_entropy(m(x).float(), y)
    loss.backward()
    return loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()}


def summary(tag, ga, gb):
    cs = [F.cosine_similarity(ga[n].flatten(), gb[n].flatten(), dim=0).item() for n in ga if gb[n].norm() > 0]
    cs.sort()
    print(f"{tag:28s} min {cs[0]:.4f}  p10 {cs[len(cs) // 10]:.4f}  median {cs[len(cs) // 2]:.4f}")


for name in ("resnet50", "resnet18"):
    torch.manual_seed(0)
    m = cast_model(build_model(name, num_classes=100).cuda().to(memory_format=torch.channels_last))
    m.train()
    x = torch.randn(32, 3, 64, 64, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 100, (32,), device="cuda")
    st = copy.deepcopy(m.state_dict())
    la, ga = grads(m, x, y)
    m.load_state_dict(st)
    conv_igemm.ENABLED = False
    lb, gb = grads(m, x, y)
    m.load_state_dict(st)
    xp = (x.float() * (1 + 2 ** -8 * torch.randn_like(x.float()))).bfloat16()
    lc, gc = grads(m, xp, y)
    m.load_state_dict(st)
    ld, gd = grads(m, x, y)
    conv_igemm.ENABLED = True
    print(name, "losses", la, lb, lc, ld)
    summary("igemm vs miopen", ga, gb)
    summary("miopen vs miopen+1ulp input", gb, gc)
    summary("miopen vs miopen (rerun)", gb, gd)
