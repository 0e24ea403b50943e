#!/usr/bin/env python3
"""Diagnostics for the flagship training step on one GPU:
host-enqueue vs device time per step, cProfile of the host side, and the
hipGraph-captured step.  Not part of the framework API."""
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
from distributed_model_parallel_amd.train.graphed import GraphedStep  # noqa: E402
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.env import init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--profile", type=int, default=1)
    a = ap.parse_args()
    env = init_distributed()
    st = build_train_state(StepConfig(model=a.model, batch_size=a.batch_size), env.device)
    for _ in range(5):
        st.step()
    torch.cuda.synchronize()
    cpu, tot = [], []
    for _ in range(10):
        t0 = time.perf_counter()
        st.step()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        cpu.append(t1 - t0)
        tot.append(t2 - t0)
    print(f"eager: host enqueue {1e3 * sum(cpu) / 10:.1f} ms/step, step {1e3 * sum(tot) / 10:.1f} ms/step",
          flush=True)
    # pipelined eager (no per-step sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        st.step()
    torch.cuda.synchronize()
    print(f"eager pipelined: {1e3 * (time.perf_counter() - t0) / 10:.1f} ms/step", flush=True)
    if a.profile:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(3):
            st.step()
        torch.cuda.synchronize()
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue()[:6000], flush=True)
    if a.graph:
        try:
            gs = GraphedStep(st.step, warmup=2)
            gs.capture()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                loss = gs()
            torch.cuda.synchronize()
            print(f"graphed: {1e3 * (time.perf_counter() - t0) / 20:.1f} ms/step loss={loss.item():.4f}",
                  flush=True)
        except Exception as e:  # noqa: BLE001
            import traceback
            traceback.print_exc()
            print(f"graph capture failed: {e!r}", flush=True)


if __name__ == "__main__":
    main()
