#!/bin/bash
# stride-2 phase dgrad (conv_xl) + c128 numerics, per-call timing, whole step
set -o pipefail
mkdir -p gpurun_out/r3j
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_igemm.py tests/test_gpu_conv_halo.py > gpurun_out/r3j/test.log 2>&1 &&
timeout -k 10 300 python -u tools/conv_roofline.py --batch 2048 --only l2.b0.conv2,l2.bN.conv2,l3.b0.conv2,l4.b0.conv2 > gpurun_out/r3j/roof.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3j/bench.log 2>&1
