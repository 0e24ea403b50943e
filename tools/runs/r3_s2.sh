#!/bin/bash
set -u
O=gpurun_out/r3g; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad3x3.py tests/test_gpu_conv_igemm.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/wgrad_bench.py --batch 2048 > $O/bench.log 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/step.log 2>&1; rc=$?; tail -1 $O/step.log; exit $rc
