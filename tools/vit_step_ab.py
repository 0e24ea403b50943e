#!/usr/bin/env python3
"""ViT-B/16 training step (DDP world 1, bf16, synthetic 224px) in three
configurations: every linear on hipBLASLt (+ separate GELU / add passes);
weight gradients on our ping-pong TN kernel (ops/linear.py _wgrad); and in
addition the MLP / projection on the fused gemm_xl epilogues (set_xl_linear).
Alternates the configurations so clock drift hits all; ms per step (HIP events).

  python tools/vit_step_ab.py [--batch 256] [--steps 10] [--rounds 2]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd.ops import linear  # noqa: E402
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.env import init_distributed, destroy_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    env = init_distributed()
    st = build_train_state(StepConfig(model="vit_b_16", batch_size=args.batch), env.device)
    cfgs = [("library", False, False), ("tn wgrad", True, False), ("tn wgrad + xl epilogues", True, True)]
    res = {c[0]: [] for c in cfgs}
    for _ in range(args.rounds):
        for name, tn, xl in cfgs:
            linear._TN_WGRAD = tn
            linear.set_xl_linear(xl)
            for _ in range(3):
                st.step()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n0, t0 = linear._STATS["xl"], linear._STATS["tn_wgrad"]
            a.record()
            for _ in range(args.steps):
                st.step()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / args.steps
            assert (linear._STATS["xl"] > n0) == xl and (linear._STATS["tn_wgrad"] > t0) == tn, \
                "linear routing did not follow the switch"
            res[name].append(ms)
            print(f"{name}: {ms:.2f} ms/step {args.batch / ms * 1e3:.0f} img/s", flush=True)
    linear.set_xl_linear(False)
    linear._TN_WGRAD = True
    print("best: " + ", ".join(f"{k} {min(v):.2f} ms" for k, v in res.items()))
    destroy_distributed()


if __name__ == "__main__":
    main()
