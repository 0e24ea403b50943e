#!/bin/bash
# kernel trace of the split-K tail probe (which of the three launches costs)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
export DMP_XL_TAIL=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r4al_prof -o prof --output-format csv -- python3 tools/tile_tail_probe.py > gpurun_out/r4al.log 2>&1
