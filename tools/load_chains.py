#!/usr/bin/env python3
"""Serialized-load scanner: compiles HIP sources to gfx950 ISA and counts, per
kernel, the vector-memory loads and the `s_waitcnt vmcnt(0)` that drain
exactly ONE outstanding load.  Such a wait right after a single load is a full
memory round trip with nothing else in flight -- the signature of a load
issued under a per-lane / per-column branch (the compiler waits for it before
the join) or of a use placed before the next load is issued.  A kernel with
many of them is latency-bound no matter its byte count (finding 67:
depthwise conv 18-31 per kernel, LayerNorm forward 8 per row).

usage: python tools/load_chains.py [csrc/conv/depthwise.hip ...] [--min 3] > profiles/load_chains.md
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def isa(src: str, out: str) -> bool:
    import torch
    tdir = os.path.dirname(torch.__file__)
    flags = ["--offload-arch=gfx950", "-x", "hip", "-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1",
             "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1", "-DTORCH_EXTENSION_NAME=_C",
             "-DTORCH_API_INCLUDE_EXTENSION_H", f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include",
             "-I/usr/include/python3.10", f"-I{os.path.join(ROOT, 'csrc')}", "--offload-device-only", "-S"]
    r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, src, "-o", out], capture_output=True, text=True)
    if r.returncode:
        print(f"<!-- {src}: compile failed: {r.stderr[-300:]} -->", file=sys.stderr)
    return r.returncode == 0


def scan(path: str):
    """-> {kernel: [loads, single-load vmcnt(0) waits, all vmcnt(0) waits with loads pending]}"""
    out, fn, pend = {}, None, 0
    with open(path) as f:
        for line in f:
            m = re.match(r"^(_Z\w+):", line)
            if m:
                fn, pend = m.group(1), 0
                out[fn] = [0, 0, 0]
                continue
            if fn is None:
                continue
            t = line.strip()
            if t.startswith(("global_load", "buffer_load")):
                out[fn][0] += 1
                pend += 1
            elif t.startswith("s_waitcnt") and "vmcnt(0)" in t:
                out[fn][1] += pend == 1
                out[fn][2] += pend > 0
                pend = 0
            elif t.startswith("s_endpgm"):
                fn = None
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("sources", nargs="*")
    ap.add_argument("--min", type=int, default=3, help="list kernels with at least this many single-load waits")
    a = ap.parse_args()
    srcs = a.sources or sorted(os.path.join(d, f) for d, _, fs in os.walk(os.path.join(ROOT, "csrc"))
                               for f in fs if f.endswith(".hip"))
    print("| source | kernel | loads | single-load vmcnt(0) waits | vmcnt(0) waits |\n|---|---|---|---|---|")
    with tempfile.TemporaryDirectory() as td:
        for src in srcs:
            s = os.path.join(td, os.path.basename(src) + ".s")
            if not isa(src, s):
                continue
            for k, (n, single, waits) in sorted(scan(s).items(), key=lambda kv: -kv[1][1]):
                if single >= a.min:
                    print(f"| {os.path.relpath(src, ROOT)} | `{k[:80]}` | {n} | {single} | {waits} |", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
