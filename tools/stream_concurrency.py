#!/usr/bin/env python3
"""How much do kernels on different streams / queues actually overlap?

Reads a rocprofv3 ``--kernel-trace --output-format csv`` directory, takes the
last complete training step (delimited by the fused-SGD kernel, as
tools/prof_summary.py) and reports: the step span, the sum of kernel
durations, the union of busy time (any kernel running), the time with two or
more kernels running, and per queue the kernel time and the part of it that
ran beside a kernel of another queue.  Used for the weight-gradient side
stream (ops/wgrad_stream.py): a large "overlapped" share with no change in
span means the two queues only time-slice the CUs.

usage: python tools/stream_concurrency.py gpurun_out/prof_x/<host>/ [--marker sgd_flat]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import sys


def load(path: str):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    return rows


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--marker", default="sgd_flat")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        print("no kernel_trace.csv under", a.dir, file=sys.stderr)
        return 1
    rows = load(files[0])
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
        st = r.get("Stream_Id", q)
        ks.append((s, e, r["Kernel_Name"], q, st))
    ks.sort()
    marks = [i for i, k in enumerate(ks) if a.marker in k[2]]
    # one optimizer launch per dtype group: keep the first of each run of markers
    marks = [m for j, m in enumerate(marks) if j == 0 or m - marks[j - 1] > 8]
    if len(marks) < 2:
        print("fewer than two step markers", file=sys.stderr)
        return 1
    lo, hi = marks[-2] + 1, marks[-1] + 1
    step = ks[lo:hi]
    t0, t1 = step[0][0], max(k[1] for k in step)
    ev = []
    for s, e, _n, q, _st in step:
        ev.append((s, 1, q))
        ev.append((e, -1, q))
    ev.sort()
    active = collections.Counter()
    busy = multi = 0
    last = ev[0][0]
    per_q_time = collections.Counter()
    per_q_over = collections.Counter()
    for t, d, q in ev:
        dt = t - last
        n = sum(active.values())
        if n >= 1:
            busy += dt
        if n >= 2:
            multi += dt
        qs = [k for k, v in active.items() if v > 0]
        for k in qs:
            per_q_time[k] += dt
            if len(qs) >= 2:
                per_q_over[k] += dt
        active[q] += d
        last = t
    total = sum(e - s for s, e, *_ in step)
    print(f"# Kernel concurrency across queues (last step: {len(step)} kernels)\n")
    print(f"| quantity | ms |\n|---|---|")
    print(f"| step span (first start .. last end) | {(t1 - t0) / 1e6:.3f} |")
    print(f"| sum of kernel durations | {total / 1e6:.3f} |")
    print(f"| busy (any kernel running) | {busy / 1e6:.3f} |")
    print(f"| two or more queues running | {multi / 1e6:.3f} |")
    print(f"| idle inside the span | {(t1 - t0 - busy) / 1e6:.3f} |")
    print("\n| queue | kernels | kernel time ms | beside another queue ms |\n|---|---|---|---|")
    cnt = collections.Counter(k[3] for k in step)
    for q, n in cnt.most_common():
        print(f"| {q} | {n} | {per_q_time[q] / 1e6:.3f} | {per_q_over[q] / 1e6:.3f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
