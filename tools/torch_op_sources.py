#!/usr/bin/env python3
"""Which Python lines launch the stock-PyTorch kernels of a training step
(copies, casts, fills, flips, cats): torch.profiler with stacks over a few
bench steps, aggregated per (aten op, innermost framework source line).

usage: python tools/torch_op_sources.py [--model resnet50] [--batch-size 256] [--steps 3]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

OPS = ("aten::copy_", "aten::to", "aten::_to_copy", "aten::fill_", "aten::zero_", "aten::flip", "aten::cat",
       "aten::stack", "aten::contiguous", "aten::clone", "aten::sum", "aten::mean", "aten::cumsum", "aten::mm",
       "aten::addmm", "aten::matmul", "aten::mul", "aten::add", "aten::sub", "aten::div", "aten::index")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from distributed_model_parallel_amd.train.step import StepConfig, build_train_state
    from distributed_model_parallel_amd.utils.env import init_distributed
    init_distributed()
    st = build_train_state(StepConfig(model=a.model, batch_size=a.batch_size), torch.device("cuda", 0))
    for _ in range(3):
        st.step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(a.steps):
            st.step()
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for ev in prof.events():
        if ev.name not in OPS or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        src = "?"
        for fr in (ev.stack or []):
            if "distributed_model_parallel_amd" in fr or "bench.py" in fr:
                src = fr.replace(root + "/", "")
                break
        if src == "?":  # no Python frame (autograd thread / C++): the enclosing ops instead
            chain, par = [], ev.cpu_parent
            while par is not None and len(chain) < 3:
                chain.append(par.name[:60])
                par = par.cpu_parent
            src = " < ".join(chain) or "?"
        key = (ev.name, src)
        agg[key][0] += 1
        agg[key][1] += sum(k.duration for k in getattr(ev, "kernels", []))
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"| aten op | source | calls/step | device us/step |\n|---|---|---|---|")
    for (name, src), (n, us) in rows[:40]:
        print(f"| {name} | {src} | {n / a.steps:.1f} | {us / a.steps:.1f} |")
    from distributed_model_parallel_amd.utils.env import destroy_distributed
    destroy_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
