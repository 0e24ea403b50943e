#!/usr/bin/env python3
"""Whole-step roofline of the bench training step (assign every
kernel of the step its bound and achieved fraction).

Builds the bench state (bench.py defaults: ResNet-50 DDP bf16 channels-last,
2048 per GPU; or --model vit_b_16 at 256), times the plain step with HIP
events, then runs ONE step with every native entry point timed in isolation
(utils/roofline.py: synchronize + events per call) and priced
(FLOPs / 2.5 PF/s vs bytes / 8 TB/s).  Prints a markdown table grouped by
(entry point, operand shapes): calls, measured ms, GFLOP, GB, bound ms,
bound type, achieved fraction; then the step summary: sum of measured, sum of
bounds, and the remainder of the plain step (library kernels, torch ops,
launch gaps).

usage: python tools/step_roofline.py [--model resnet50] [--batch-size 2048] > profiles/x.md
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    from distributed_model_parallel_amd.train.step import StepConfig, build_train_state
    from distributed_model_parallel_amd.utils import gemm_tuning, miopen_db, roofline
    from distributed_model_parallel_amd.utils.env import destroy_distributed, init_distributed
    bs = a.batch_size or {"resnet50": 2048, "vit_b_16": 256}.get(a.model, 256)
    env = init_distributed()
    miopen_db.seed("use")
    gemm_tuning.configure("use", a.model)
    st = build_train_state(StepConfig(model=a.model, batch_size=bs), env.device)
    for _ in range(3):
        st.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        st.step()
    e1.record()
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / a.steps
    with roofline.probe() as p:
        st.step()
        torch.cuda.synchronize()
    rows = roofline.aggregate(p.records)
    tot_ms = sum(r["ms"] for r in rows)
    tot_bound = sum(r["bound_ms"] for r in rows)
    tot_f = sum(r["gflop"] for r in rows)
    print(f"# Step roofline: {a.model}, batch {bs}, 1x MI355X\n")
    print(f"Plain step (HIP events, mean of {a.steps}): **{step_ms:.2f} ms**.  Probed native calls: "
          f"{len(p.records)} in {len(rows)} groups, **{tot_ms:.2f} ms** measured in isolation, "
          f"roofline bound **{tot_bound:.2f} ms** ({tot_bound / tot_ms:.0%} of measured; "
          f"{tot_f / 1e3:.1f} TFLOP -> {tot_f / tot_ms:.0f} TF/s average).  Not probed (library / torch "
          f"kernels, launch gaps): {step_ms - tot_ms:.2f} ms.\n")
    print("Bound = max(FLOP / 2.5 PF/s, bytes / 8 TB/s); bytes = operands read once + results written once "
          "(a lower bound).  frac = bound / measured.\n")
    print("| entry point | leading operand shapes | calls | ms | GFLOP | GB | bound ms | bound | frac |")
    print("|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        shp = " ".join("x".join(str(d) for d in s) for s in r["shapes"])
        print(f"| `{r['fn']}` | {shp} | {r['calls']} | {r['ms']:.3f} | {r['gflop']:.1f} | {r['gb']:.2f} | "
              f"{r['bound_ms']:.3f} | {r['bound']} | {r['frac']:.0%} |")
    by = {}
    for r in rows:
        d = by.setdefault(r["fn"], [0.0, 0.0])
        d[0] += r["ms"]
        d[1] += r["bound_ms"]
    print("\n| entry point | ms | bound ms | frac |\n|---|---|---|---|")
    for fn, (ms, b) in sorted(by.items(), key=lambda kv: -kv[1][0]):
        print(f"| `{fn}` | {ms:.3f} | {b:.3f} | {b / ms:.0%} |")
    destroy_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
