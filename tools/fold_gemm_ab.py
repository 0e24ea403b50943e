#!/usr/bin/env python3
"""ResNet-50 training step (DDP world 1, bf16, synthetic) with the BN-fold
coefficient products (W G forward; W^T diag(be) W and c^T W backward) on
hipBLASLt fp32 GEMMs (set_fold_gemm(1)) vs our fp32-MFMA tiled kernel
(set_fold_gemm(2)).  Alternates the modes so clock drift hits both; ms per
step (HIP events around --steps steps).

  python tools/fold_gemm_ab.py [--batch 2048] [--steps 10] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.env import destroy_distributed, init_distributed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="1,2")
    a = ap.parse_args()
    env = init_distributed()
    C = _native.require("fold gemm A/B")
    st = build_train_state(StepConfig(model="resnet50", batch_size=a.batch), env.device)
    modes = [int(m) for m in a.modes.split(",")]
    old = C.get_fold_gemm()
    times = {m: [] for m in modes}
    try:
        for m in modes:  # warm every mode once
            C.set_fold_gemm(m)
            for _ in range(3):
                st.step()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for m in modes:
                C.set_fold_gemm(m)
                st.step()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.steps):
                    st.step()
                e1.record()
                torch.cuda.synchronize()
                times[m].append(e0.elapsed_time(e1) / a.steps)
    finally:
        C.set_fold_gemm(old)
    for m in modes:
        print(f"fold_gemm {m}: {statistics.median(times[m]):.3f} ms/step (runs {', '.join(f'{t:.3f}' for t in times[m])})",
              flush=True)
    destroy_distributed()


if __name__ == "__main__":
    main()
