#!/usr/bin/env python3
"""A few launches of the halo-tiled 3x3 conv (forward store, batch 1024) for a
rocprofv3 --pmc pass:

  timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS \\
      SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_LDS \\
      -d gpurun_out/halo_pmc -- python3 tools/halo_pmc.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_model_parallel_amd import _native  # noqa: E402
from distributed_model_parallel_amd.ops import conv_igemm  # noqa: E402

C = _native.require("halo pmc")
x = torch.randn(1024, 64, 56, 56, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(64, 64, 3, 3, device="cuda") / 24).bfloat16().contiguous(memory_format=torch.channels_last)
wm = conv_igemm._wmat(w).contiguous()
for _ in range(3):
    C.conv3x3_c64(x, wm, False)
torch.cuda.synchronize()
print("done")
