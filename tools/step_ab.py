#!/usr/bin/env python3
"""In-step A/B of kernel routing choices on one box (DDP world 1, bf16,
synthetic data, the bench step of train/step.py).  Arms are applied by
setters, alternated round by round so clock drift hits all; ms per step from
HIP events around --steps steps after 3 untimed ones.

arms:
  bm256      4-wave GEMMs always on 256-row tiles (_C.set_gemm_xl_bm(-1))
  bmauto     224-row tiles where they fill the last round (pick_bm_w4, default)
  bm224      224-row tiles for every 4-wave GEMM
  plain_lib  ViT plain GEMMs (qkv forward, N = 768 data gradients) on hipBLASLt
  plain_fwd  qkv forward on gemm_xl, data gradients on hipBLASLt
  plain_xl   every plain GEMM on gemm_xl
  fold1 / fold2  BN-fold coefficient products on hipBLASLt / our fp32 MFMA GEMM
  flipc / flipt  3x3 data-gradient weights flipped once per optimizer step (cache) / per backward (torch)
  tnmin16k / 8k / 4k  row threshold of the 4-wave TN weight gradients (below: the split-M gemm_tn kernel)
  tnch64 / tnch16  narrowest 1x1 weight-gradient side on the 4-wave TN kernel
  trimh / notrimh  trimmed row tiles for the PIPE-10 heavy-epilogue (short-K) GEMMs / 256 rows
  f32c / f32t  BN-fold fp32 weights from the optimizer-driven cache / a cast per forward
  finf / finsep  BN-fold finalize fused into the folded-moments launch / a separate bn_finalize
  tnnarrow / tnwide  4-wave weight gradients with a side of 64 / 128 on narrow tiles / on 256 x 256
  n128 / miopen  Cout = 128 3x3 forwards (ResNet-50 layer-2 stride 2) on the 4-wave 256 x 128 tile / MIOpen

  python tools/step_ab.py --model vit_b_16 --batch 256 --arms plain_fwd,plain_xl [--steps 10] [--rounds 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops import bn_fold, conv1x1, conv_igemm, linear, wt_cache  # noqa: E402
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.env import init_distributed, destroy_distributed  # noqa: E402


_AS_F32 = [None]


def _plain(mode):
    def f():
        linear._PLAIN_LIB = mode == "lib"
        linear._PLAIN_FWD_XL = mode in ("xl", "fwd")
        linear._PLAIN_DGRAD_XL = mode == "xl"
    return f


def _arm(name):
    C = _native.native()
    table = {
        "bm256": lambda: C.set_gemm_xl_bm(-1),
        "bmauto": lambda: C.set_gemm_xl_bm(0),
        "bm224": lambda: C.set_gemm_xl_bm(224),
        "plain_lib": _plain("lib"),
        "plain_fwd": _plain("fwd"),
        "plain_xl": _plain("xl"),
        "fold1": lambda: C.set_fold_gemm(1),
        "fold2": lambda: C.set_fold_gemm(2),
        "n128": lambda: setattr(conv_igemm, "_XL_N128", True),
        "miopen": lambda: setattr(conv_igemm, "_XL_N128", False),
        "flipc": lambda: wt_cache._FLIP.__setitem__(0, True),
        "flipt": lambda: wt_cache._FLIP.__setitem__(0, False),
        "tnmin16k": lambda: setattr(conv1x1, "_TN_XL_MIN_ROWS", 16384),
        "tnmin8k": lambda: setattr(conv1x1, "_TN_XL_MIN_ROWS", 8192),
        "tnmin4k": lambda: setattr(conv1x1, "_TN_XL_MIN_ROWS", 4096),
        "tnch64": lambda: setattr(conv1x1, "_TN_XL_MIN_CH", 64),
        "tnch16": lambda: setattr(conv1x1, "_TN_XL_MIN_CH", 16),
        "trimh": lambda: C.set_gemm_xl_trim_heavy(True),
        "notrimh": lambda: C.set_gemm_xl_trim_heavy(False),
        "f32c": lambda: setattr(wt_cache, "as_f32", _AS_F32[0]),
        "f32t": lambda: setattr(wt_cache, "as_f32", lambda w: None),
        "finf": lambda: setattr(bn_fold, "_FUSED_FINALIZE", True),
        "finsep": lambda: setattr(bn_fold, "_FUSED_FINALIZE", False),
        "tnnarrow": lambda: C.set_tn_narrow(True),
        "tnwide": lambda: C.set_tn_narrow(False),
    }
    return table[name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--arms", default="bm256,bmauto")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    _AS_F32[0] = wt_cache.as_f32
    env = init_distributed()
    st = build_train_state(StepConfig(model=args.model, batch_size=args.batch), env.device)
    arms = args.arms.split(",")
    res = {a: [] for a in arms}
    for r in range(args.rounds):
        for a in (arms if r % 2 == 0 else arms[::-1]):
            _arm(a)()
            for _ in range(3):
                st.step()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.steps):
                st.step()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / args.steps
            res[a].append(ms)
            print(f"round {r} {a}: {ms:.3f} ms/step", flush=True)
    print(f"{args.model} batch {args.batch}: " +
          ", ".join(f"{a} median {sorted(v)[len(v) // 2]:.3f} min {min(v):.3f} ms" for a, v in res.items()))
    destroy_distributed()


if __name__ == "__main__":
    main()
