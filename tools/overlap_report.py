#!/usr/bin/env python3
"""Communication / compute overlap from a rocprofv3 kernel trace.

For every collective kernel (RCCL) in the last complete training step:
start, duration, the share of its lifetime during which a compute kernel was
also running on the device, and the "exposed" communication time after the
last compute kernel of the step.  Steps are delimited by the fused-SGD kernel
(one launch per dtype group, tools/prof_summary.py convention).

On one GPU run the bench with ``DMP_DDP_SINGLE_RANK_COMM=1`` so the DDP reducer
really issues its bucket all-reduces through RCCL (a world-size-1 RCCL
all-reduce is still a device kernel on the communicator's stream): the trace
then shows where each bucket's collective sits relative to the backward.

usage: python tools/overlap_report.py gpurun_out/prof_dir/<host>/ > profiles/x.md
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import sys

COMM_KEYS = ("nccl", "rccl", "oneRank", "ncclDevKernel")


def is_comm(name: str) -> bool:
    return any(k in name for k in COMM_KEYS)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="sgd_flat")
    ap.add_argument("--title", default="DDP bucket all-reduce overlap")
    a = ap.parse_args()
    trace = glob.glob(os.path.join(a.dir, "*kernel_trace.csv"))
    if not trace:
        print("no kernel_trace.csv in", a.dir, file=sys.stderr)
        return 1
    rows = list(csv.DictReader(open(trace[0])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    bounds = []
    for i in marks:
        if not bounds or i - bounds[-1] > 4:
            bounds.append(i)
        else:
            bounds[-1] = i
    if len(bounds) < 2:
        print("fewer than two step markers found", file=sys.stderr)
        return 1
    seg = rows[bounds[-2] + 1: bounds[-1] + 1]
    comm = [r for r in seg if is_comm(r["Kernel_Name"])]
    comp = [r for r in seg if not is_comm(r["Kernel_Name"])]
    t0 = seg[0]["s"]
    # merged busy intervals of compute kernels
    iv = sorted((r["s"], r["e"]) for r in comp)
    merged = []
    for s, e in iv:
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])

    def overlap(s, e):
        tot = 0
        for ms, me in merged:
            if me <= s:
                continue
            if ms >= e:
                break
            tot += min(e, me) - max(s, ms)
        return tot

    # last backward compute kernel before the optimizer: everything before the marker
    opt_start = min(r["s"] for r in seg if a.marker in r["Kernel_Name"])
    bwd_end = max((r["e"] for r in comp if r["e"] <= opt_start), default=opt_start)
    print(f"# {a.title}\n")
    print(f"step span {(seg[-1]['e'] - t0) / 1e6:.2f} ms, {len(comp)} compute kernels, "
          f"{len(comm)} collective kernels\n")
    print("| # | start (ms into step) | duration us | overlapped with compute % | kernel |")
    print("|---|---|---|---|---|")
    tot_d = tot_o = 0
    exposed = 0
    for i, r in enumerate(comm):
        d = r["e"] - r["s"]
        o = overlap(r["s"], r["e"])
        tot_d += d
        tot_o += o
        if r["e"] > bwd_end:
            exposed += r["e"] - max(r["s"], bwd_end)
        print(f"| {i} | {(r['s'] - t0) / 1e6:.2f} | {d / 1e3:.1f} | {100 * o / max(d, 1):.0f} | "
              f"`{r['Kernel_Name'][:60]}` |")
    if comm:
        print(f"\ncollective time {tot_d / 1e3:.1f} us, {100 * tot_o / max(tot_d, 1):.0f} % of it "
              f"concurrent with compute kernels; {exposed / 1e3:.1f} us after the last backward "
              f"compute kernel (exposed before the optimizer step).")
    return 0


if __name__ == "__main__":
    sys.exit(main())
