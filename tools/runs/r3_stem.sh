#!/bin/bash
set -u
O=gpurun_out/r3f; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/stem_bench.py --batch 2048 > $O/bench.log 2>&1; rc=$?; grep -v amdgpu.ids $O/bench.log; exit $rc
