#!/bin/bash
# tests of the conv paths, then the headline bench and a kernel trace of it
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3d; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_wgrad3x3.py tests/test_gpu_conv_igemm.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1; rc=$?; tail -3 $O/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --steps 6 --warmup 2 > $O/prof.log 2>&1; rc=$?; tail -1 $O/prof.log; exit $rc
