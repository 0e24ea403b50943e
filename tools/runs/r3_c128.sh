#!/bin/bash
# conv3x3_c128: numerics, per-call timing vs MIOpen, whole-step bench
set -o pipefail
mkdir -p gpurun_out/r3i
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_conv_halo.py tests/test_halo_layout.py > gpurun_out/r3i/test.log 2>&1 &&
timeout -k 10 180 python -u tools/halo_bench.py --batch 2048 --c 128 > gpurun_out/r3i/halobench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3i/bench.log 2>&1
