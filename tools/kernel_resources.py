#!/usr/bin/env python3
"""Per-kernel register / scratch / LDS / occupancy table for every HIP source
(hipcc -Rpass-analysis=kernel-resource-usage, gfx950), as markdown.  Exits 1
if any kernel spills to scratch (a dynamically indexed register array -- see
csrc/conv/depthwise.hip -- or register pressure): that is a silent 2-4x.

usage: python tools/kernel_resources.py > profiles/kernel_resources.md
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "csrc"))


def _flags():
    import torch
    tdir = os.path.dirname(torch.__file__)
    return ["--offload-arch=gfx950", "-x", "hip", "-munsafe-fp-atomics", "-O3", "-fPIC", "-std=c++17",
            "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-D_GLIBCXX_USE_CXX11_ABI=1",
            "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
            f"-I{tdir}/include", f"-I{tdir}/include/torch/csrc/api/include", "-I/usr/include/python3.10",
            "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"]


def resources(src: str) -> list:
    """Per-kernel resource dicts of one HIP source: name (demangled, no
    namespace), VGPR, AGPR, scratch (bytes/lane), lds, occupancy."""
    r = subprocess.run(["/opt/rocm/bin/hipcc", *_flags(), "-c", src, "-o", "/dev/null"],
                       capture_output=True, text=True)
    out, cur = [], {}
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        kv = m.group(1)
        if kv.startswith("Function Name:"):
            cur = {"name": kv.split(":", 1)[1].strip()}
        elif ":" in kv:
            k, v = kv.split(":", 1)
            cur[k.strip()] = v.strip()
            if k.strip().startswith("LDS Size"):
                name = subprocess.run(["c++filt", cur["name"]], capture_output=True, text=True).stdout.strip()
                name = name.replace("dmp::(anonymous namespace)::", "").replace("void ", "")
                name = re.sub(r"\(.*", "", name)
                out.append({"name": name, "vgpr": cur.get("VGPRs", "?"), "agpr": cur.get("AGPRs", "?"),
                            "scratch": cur.get("ScratchSize [bytes/lane]", "?"), "lds": v.strip(),
                            "occupancy": cur.get("Occupancy [waves/SIMD]", "?")})
    return out


def main() -> int:
    srcs = []
    for d, _, fs in os.walk(os.path.join(ROOT, "csrc")):
        srcs += [os.path.join(d, f) for f in fs if f.endswith(".hip")]
    bad = 0
    print("| source | kernel | VGPR | AGPR | scratch B/lane | LDS B | waves/SIMD |\n|---|---|---|---|---|---|---|")
    for src in sorted(srcs):
        for k in resources(src):
            bad += k["scratch"] not in ("0", "?")
            print(f"| {os.path.relpath(src, ROOT)} | `{k['name'][:90]}` | {k['vgpr']} | {k['agpr']} | "
                  f"{k['scratch']} | {k['lds']} | {k['occupancy']} |")
    print(f"\nkernels with scratch: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
