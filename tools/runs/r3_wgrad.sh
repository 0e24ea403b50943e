#!/bin/bash
set -u
O=gpurun_out/r3b; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad3x3.py -x -v --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -15 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/conv_roofline.py --batch 2048 --only l1.bN.conv2,l2.bN.conv2,l3.bN.conv2,l4.bN.conv2 > $O/roof.log 2>&1; rc=$?; cat $O/roof.log | grep -v amdgpu.ids; exit $rc
