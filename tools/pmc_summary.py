#!/usr/bin/env python3
"""Per-kernel summary of rocprofv3 --pmc counter CSVs: mean value per dispatch
of every counter, for the kernels whose name contains a filter string.

usage: python tools/pmc_summary.py <dir-or-csv> [<dir-or-csv> ...] [--match attn_] [--skip 1]
(--skip drops each kernel's first N dispatches: warm-up / code-object load)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--skip", type=int, default=1)
    a = ap.parse_args()
    files = []
    for p in a.paths:
        files += glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True) if os.path.isdir(p) else [p]
    # kernel -> counter -> dispatch id -> value (a dispatch can be split per XCD / SE rows: summed)
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                if a.match and a.match not in r["Kernel_Name"]:
                    continue
                k = short(r["Kernel_Name"])
                vals[k][r["Counter_Name"]][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
    for k, cs in sorted(vals.items()):
        print(f"### {k}\n\n| counter | mean per dispatch | dispatches |\n|---|---|---|")
        for c, d in sorted(cs.items()):
            v = [d[key] for key in sorted(d)][a.skip:] or list(d.values())
            print(f"| {c} | {sum(v) / len(v):,.0f} | {len(v)} |")
        print()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
