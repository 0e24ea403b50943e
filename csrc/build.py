#!/usr/bin/env python3
"""Build the native extension ``distributed_model_parallel_amd/_C.so`` for gfx950.

No hipify, no cpp_extension JIT: ``.hip`` sources go straight through
``hipcc --offload-arch=gfx950``; host ``.cpp`` sources through ``g++`` (the
compiler PyTorch itself is built with, so the C++ ABI matches); the objects are
linked against the HIP runtime and RCCL that PyTorch already loads (its own
``torch/lib`` copies, so one process never holds two RCCL/HIP runtimes).

Incremental: an object is rebuilt when its source or any header under csrc/
is newer.  Usage: ``python csrc/build.py [-j N] [--force] [--asan]``.

``--asan`` (host code only -- GPU AddressSanitizer is not
available here): every object is rebuilt with ``-fsanitize=address`` on the
HOST side (``-Xarch_host`` for hipcc, device code untouched) into
``build/native-asan/_C.so``; run the CPU suite against it with::

    LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libstdc++.so)" \
        ASAN_OPTIONS=detect_leaks=0 DMP_NATIVE_SO=build/native-asan/_C.so python -m pytest tests -m "not gpu"
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
PKG = ROOT / "distributed_model_parallel_amd"
OUT = PKG / "_C.so"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("DMP_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch  # noqa: WPS433
    tdir = Path(torch.__file__).resolve().parent
    inc = [tdir / "include", tdir / "include" / "torch" / "csrc" / "api" / "include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return tdir, inc, abi


def sources():
    hip = sorted(CSRC.rglob("*.hip"))
    cpp = sorted(CSRC.rglob("*.cpp"))
    return hip, cpp


def _newest_header() -> float:
    hs = list(CSRC.rglob("*.h")) + list(CSRC.rglob("*.hpp"))
    return max((h.stat().st_mtime for h in hs), default=0.0)


def _obj_for(src: Path) -> Path:
    rel = src.relative_to(CSRC)
    return BUILD / (str(rel).replace(os.sep, "__") + ".o")


def _common_flags(inc, abi):
    py_inc = sysconfig.get_paths()["include"]
    flags = [
        "-O3", "-fPIC", "-std=c++17",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-I{py_inc}", f"-I{ROCM / 'include'}", f"-I{CSRC}",
    ]
    for p in inc:
        flags.append(f"-isystem{p}")
    return flags


ASAN = False


def _obj_for_build(src: Path) -> Path:
    o = _obj_for(src)
    return (ROOT / "build" / "native-asan" / o.name) if ASAN else o


def compile_one(src: Path, inc, abi, force: bool, hdr_mtime: float) -> tuple[Path, str]:
    obj = _obj_for_build(src)
    if not force and obj.exists():
        m = obj.stat().st_mtime
        if m >= src.stat().st_mtime and m >= hdr_mtime:
            return obj, "up-to-date"
    obj.parent.mkdir(parents=True, exist_ok=True)
    common = _common_flags(inc, abi)
    if src.suffix == ".hip":
        san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fno-omit-frame-pointer"] if ASAN else []
        cmd = [str(ROCM / "bin" / "hipcc"), f"--offload-arch={ARCH}", "-x", "hip",
               "-munsafe-fp-atomics", "-Wno-unused-result", *san, *common, "-c", str(src), "-o", str(obj)]
    else:
        san = ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"] if ASAN else []
        cmd = ["g++", *common, *san, "-Wno-unused-result", "-Wno-deprecated-declarations", "-c", str(src),
               "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj, "built"


def link(objs, tdir: Path, out: Path = OUT):
    tlib = tdir / "lib"
    cmd = ["g++", "-shared", *(["-fsanitize=address"] if ASAN else []), "-o", str(out),
           *[str(o) for o in objs],
           f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
           "-ltorch_python", "-lamdhip64", "-lrccl",
           f"-Wl,-rpath,{tlib}", f"-Wl,-rpath,{ROCM / 'lib'}"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build(jobs: int = 8, force: bool = False, verbose: bool = True) -> Path:
    tdir, inc, abi = _torch_paths()
    hip, cpp = sources()
    hdr = _newest_header()
    BUILD.mkdir(parents=True, exist_ok=True)
    objs, changed = [], False
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = {ex.submit(compile_one, s, inc, abi, force, hdr): s for s in hip + cpp}
        for f in cf.as_completed(futs):
            obj, status = f.result()
            objs.append(obj)
            changed |= status == "built"
            if verbose:
                print(f"[dmp-build] {status:10s} {futs[f].relative_to(ROOT)}", flush=True)
    objs.sort()
    out = (ROOT / "build" / "native-asan" / "_C.so") if ASAN else OUT
    if changed or force or not out.exists() or out.stat().st_mtime < max(o.stat().st_mtime for o in objs):
        link(objs, tdir, out)
        if verbose:
            print(f"[dmp-build] linked {out.relative_to(ROOT)}", flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--asan", action="store_true", help="host-side AddressSanitizer build (CPU tests)")
    a = ap.parse_args()
    ASAN = a.asan
    try:
        build(a.jobs, a.force)
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
