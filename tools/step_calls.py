#!/usr/bin/env python3
"""List one training step's kernels from a rocprofv3 run (SQLite results db
or kernel-trace CSV) with grid / workgroup sizes and durations, so each call
can be matched to its GEMM shape (grid = tiles); the last step is the span
after the second-to-last fused-SGD launch.

usage: python tools/step_calls.py gpurun_out/prof_x/run_results.db [--match gemm_nt] [--top 40]
"""
import argparse
import collections
import csv
import sqlite3


def load(path):
    if path.endswith(".db"):
        cur = sqlite3.connect(path).cursor()
        q = "select name, start, end, grid_x, workgroup_x from kernels order by start"
        return [dict(zip(("name", "start", "end", "grid", "wg"), r)) for r in cur.execute(q)]
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append({"name": r["Kernel_Name"], "start": int(r["Start_Timestamp"]), "end": int(r["End_Timestamp"]),
                     "grid": r.get("Grid_Size_X", r.get("Grid_Size", "?")),
                     "wg": r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?"))})
    return sorted(rows, key=lambda r: r["start"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=0, help="group by (kernel, grid) and print the N largest")
    a = ap.parse_args()
    rows = load(a.path)
    sgd = []  # the last launch of each optimizer group (several flat buffers: one launch each)
    for i, r in enumerate(rows):
        if "sgd_flat" in r["name"]:
            if sgd and i - sgd[-1] <= 4:
                sgd[-1] = i
            else:
                sgd.append(i)
    lo = sgd[-2] + 1 if len(sgd) >= 2 else 0
    hi = sgd[-1] + 1 if sgd else len(rows)
    step = [r for r in rows[lo:hi] if a.match in r["name"]]
    if a.top:
        g = collections.defaultdict(lambda: [0, 0.0])
        for r in step:
            k = (r["name"][:100], r["grid"], r["wg"])
            g[k][0] += 1
            g[k][1] += (r["end"] - r["start"]) / 1e3
        print("| us total | calls | us/call | grid | wg | kernel |\n|---|---|---|---|---|---|")
        for k, (n, us) in sorted(g.items(), key=lambda kv: -kv[1][1])[:a.top]:
            print(f"| {us:.0f} | {n} | {us / n:.0f} | {k[1]} | {k[2]} | `{k[0]}` |")
        return
    print("| # | us | grid | wg | kernel |\n|---|---|---|---|---|")
    for i, r in enumerate(step):
        print(f"| {i} | {(r['end'] - r['start']) / 1e3:.1f} | {r['grid']} | {r['wg']} | `{r['name'][:110]}` |")


if __name__ == "__main__":
    main()
