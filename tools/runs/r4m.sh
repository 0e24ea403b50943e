#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "120|r4m_small|ONLY=cbr512,cbr512x2,cbr512x3,cb512x2_norelu,block512x2,cbr256x2_4x4,cbr64x2_16x16 VERBOSE=1 $G" \
  "120|r4m_small_noigemm|ONLY=cbr512x2,block512x2 DMP_DISABLE=igemm VERBOSE=1 $G"
