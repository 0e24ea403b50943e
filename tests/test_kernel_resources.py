"""Build-time guard for the 4-wave GEMM (gemm_xl PIPE 11): its MFMAs are
inline asm with the accumulators pinned to AGPRs, so the compiler does not
know they are still being written for ~18 cycles after each issue.  Any
compiler spill of an accumulator right behind its MFMA reads a stale value
(seen once: XL_BNBWD's epilogue pushed the kernel to 36 B of scratch and 0.2 %
of its outputs came out wrong).  Every instantiation must therefore build with
zero scratch and its accumulators in AGPRs (256; 224 for the trimmed
224-row tiles, MB = 7; 128 for the 256 x 128 tiles, MB = 4).  CPU only (hipcc
cross-compiles gfx950)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("c++filt") is None,
                    reason="needs hipcc and c++filt")
def test_w4_gemm_kernels_never_spill():
    from tools.kernel_resources import resources
    ks = [k for k in resources(os.path.join(ROOT, "csrc", "gemm", "gemm_xl.hip"))
          if k["name"].startswith(("gemm_xl_w4_kernel", "gemm_tn_w4_kernel"))]
    assert len(ks) >= 20, [k["name"] for k in ks]
    bad = [(k["name"], k["scratch"]) for k in ks if k["scratch"] != "0"]
    assert not bad, f"4-wave GEMM instantiations with scratch (accumulator spills behind asm MFMAs): {bad}"
    # trimmed 224-row tiles (template MB = 7, the last template argument) hold 56 accumulators
    # and the 256 x 128 tiles (MB = 4, WN = 1) 32
    # narrow TN tiles (gemm_tn_w4_kernel<0, TNN, TNK>): 64 x 256 / 256 x 64 hold 64,
    # 128 x 256 / 256 x 128 hold 128
    def want_agpr(name):
        n = name.replace(" ", "")
        if n.startswith("gemm_tn_w4_kernel<0,"):
            return "64" if ",64," in n or n.endswith(",64>") else "128" if ",128," in n or n.endswith(",128>") else "256"
        return "224" if n.endswith(",7,2,8>") else "128" if n.endswith(",4,1,8>") else "256"
    want = {k["name"]: want_agpr(k["name"]) for k in ks}
    assert all(int(k["agpr"]) >= int(want[k["name"]]) for k in ks), [(k["name"], k["agpr"]) for k in ks]
    assert any(want[k["name"]] == "224" for k in ks), "no trimmed (MB = 7) instantiation built"
