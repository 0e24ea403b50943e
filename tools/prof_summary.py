#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown:
per-step device time, top kernels by total time, kernel categories.

usage: python tools/prof_summary.py gpurun_out/prof_x/<host>/ [--steps-marker sgd_flat] > profiles/x.md
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import sys

CATS = [
    ("dmp BN (ours)", ("bn_moments", "bn_apply", "bn_bwd", "bn_reduce", "bn_finalize")),
    ("dmp BN fold coefficients (ours)", ("fold_fwd", "fold_bwd", "fold_coef")),
    ("dmp fused SGD (ours)", ("sgd_flat",)),
    ("dmp coalesced copy/reduce (ours)", ("multi_copy", "reduce_add", "gather_slabs")),
    ("dmp GEMM/conv (ours)", ("gemm_nt_kernel", "gemm_tn_kernel", "gemm_xl", "gemm_x2", "gemm_tn_w4", "gemm_tn_pp",
                              "split_reduce", "dw_fwd",
                              "dw_dgrad", "dw_wgrad", "column_reduce", "conv3x3_c64", "conv3x3_c128", "gemm_tn_pp",
                              "wgrad3x3", "wgrad_reduce", "stem_fwd", "stem_wgrad", "partial_sum_kernel",
                              "s2d_kernel")),
    ("dmp attention (ours)", ("attn_fwd_kernel", "attn_bwd_kernel")),
    ("dmp LayerNorm (ours)", ("ln_fwd", "ln_bwd", "ln_col_reduce")),
    ("dmp linear side passes (ours)", ("colsum_kernel", "partial_colsum")),
    ("MIOpen conv (igemm/ck)", ("igemm", "conv", "ck::", "naive_conv", "gridwise")),
    ("MIOpen tensor ops", ("SubTensorOp", "Op1dTensor", "Op2dTensor", "Op4dTensor")),
    ("hipBLASLt / rocBLAS GEMM", ("Cijk", "gemm", "Gemm")),
    ("RCCL", ("ncclDevKernel", "oneRankReduce", "nccl", "rccl")),
    ("pooling", ("pool",)),
    ("torch elementwise/reduce", ("at::native",)),
    ("runtime fill/copy", ("__amd_rocclr",)),
]


def cat_of(name: str) -> str:
    for c, keys in CATS:
        if any(k in name for k in keys):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="sgd_flat")
    ap.add_argument("--title", default="")
    ap.add_argument("--sequence", type=int, default=0,
                    help="also list the first N kernels of the last step in launch order")
    a = ap.parse_args()
    trace = glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))
    stats = glob.glob(os.path.join(a.dir, "*kernel_stats.csv"))
    rows = list(csv.DictReader(open(trace[0]))) if trace else []
    dbs = glob.glob(os.path.join(a.dir, "*_results.db"))
    if not rows and dbs:  # rocprofv3's default (rocpd sqlite) output
        import sqlite3
        con = sqlite3.connect(dbs[0])
        rows = [{"Kernel_Name": n, "Start_Timestamp": str(st), "End_Timestamp": str(en)}
                for n, st, en in con.execute("select name, start, end from kernels")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    out = sys.stdout
    if a.title:
        print(f"# {a.title}\n", file=out)
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    # group consecutive marker kernels (one per dtype group) into one step boundary
    bounds = []
    for i in marks:
        if not bounds or i - bounds[-1] > 4:
            bounds.append(i)
        else:
            bounds[-1] = i
    steps = []
    for s in range(1, len(bounds)):
        seg = rows[bounds[s - 1] + 1: bounds[s] + 1]
        span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e6
        steps.append((len(seg), span, busy, seg))
    if steps:
        print("| step | kernels | span ms | sum of kernel ms |\n|---|---|---|---|", file=out)
        for i, (n, sp, b, _) in enumerate(steps):
            print(f"| {i} | {n} | {sp:.2f} | {b:.2f} |", file=out)
        last = steps[-1][3]
        agg = collections.defaultdict(lambda: [0, 0.0])
        cats = collections.defaultdict(float)
        for r in last:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            agg[r["Kernel_Name"][:110]][0] += 1
            agg[r["Kernel_Name"][:110]][1] += d
            cats[cat_of(r["Kernel_Name"])] += d
        tot = sum(cats.values())
        print(f"\n## Last step by category (sum {tot:.2f} ms)\n\n| category | ms | % |\n|---|---|---|", file=out)
        for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
            print(f"| {c} | {v:.2f} | {100 * v / tot:.1f} |", file=out)
        print("\n## Last step, top kernels\n\n| ms | calls | kernel |\n|---|---|---|", file=out)
        for k, (n, v) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
            print(f"| {v:.3f} | {n} | `{k}` |", file=out)
        if a.sequence:
            print(f"\n## Last step, first {a.sequence} kernels in launch order\n\n| # | us | gap us | kernel |"
                  "\n|---|---|---|---|", file=out)
            prev = None
            for i, r in enumerate(last[: a.sequence]):
                st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                gap = (st - prev) / 1e3 if prev is not None else 0.0
                prev = en
                print(f"| {i} | {(en - st) / 1e3:.1f} | {gap:.1f} | `{r['Kernel_Name'][:90]}` |", file=out)
    elif stats:
        print("| ms | calls | kernel |\n|---|---|---|", file=out)
        for r in list(csv.DictReader(open(stats[0])))[:30]:
            print(f"| {float(r['TotalDurationNs']) / 1e6:.3f} | {r['Calls']} | `{r['Name'][:110]}` |", file=out)


if __name__ == "__main__":
    main()
