#!/bin/bash
# c128 stride-2 phase dgrad: numerics, per-call roofline, bench, trace (v23)
set -o pipefail
mkdir -p gpurun_out/r3k
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py tests/test_gpu_conv_igemm.py tests/test_gpu_wgrad3x3.py > gpurun_out/r3k/test.log 2>&1 &&
timeout -k 10 300 python -u tools/conv_roofline.py --batch 2048 --only l2.b0.conv2,l2.bN.conv2 > gpurun_out/r3k/roof.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3k/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3k/prof -o prof -- python -u bench.py --steps 6 --warmup 2 > gpurun_out/r3k/prof.log 2>&1
