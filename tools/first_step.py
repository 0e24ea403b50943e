#!/usr/bin/env python3
"""Where does the first (cold) training step spend its time?  cProfile of
step 0 plus per-module forward wall times (device-synchronised).  Diagnostic
only (profiles/README.md finding 9)."""
from __future__ import annotations

import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils import gemm_tuning, miopen_db  # noqa: E402
from distributed_model_parallel_amd.utils.env import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=512)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--benchmark", type=int, default=1)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    env = init_distributed()
    torch.backends.cudnn.benchmark = bool(a.benchmark)
    miopen_db.seed("use")
    gemm_tuning.configure("use", a.model)
    st = build_train_state(StepConfig(model=a.model, batch_size=a.batch_size), env.device)
    times = {}

    def pre(m, _inp):
        torch.cuda.synchronize()
        m._t0 = time.perf_counter()

    def post(m, _inp, _out):
        torch.cuda.synchronize()
        times[m._name] = time.perf_counter() - m._t0

    for name, m in st.model.named_modules():
        if name and len(list(m.children())) == 0:
            m._name = name
            m.register_forward_pre_hook(pre)
            m.register_forward_hook(post)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as prof:
        st.step()
        torch.cuda.synchronize()
    pr.disable()
    print(f"step 0: {time.perf_counter() - t0:.1f} s", flush=True)
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cpu_time_total",
                                                              row_limit=30, max_name_column_width=40,
                                                              max_shapes_column_width=90))
    for k, v in sorted(times.items(), key=lambda kv: -kv[1])[:20]:
        print(f"  fwd {v * 1e3:9.1f} ms  {k}")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())
    t0 = time.perf_counter()
    st.step()
    torch.cuda.synchronize()
    print(f"step 1: {time.perf_counter() - t0:.3f} s")


if __name__ == "__main__":
    main()
