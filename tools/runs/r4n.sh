#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "120|r4n|ONLY=bnrelu512,bn512,conv_bn_stockrelu,conv_stockrelu,conv_only,conv1x1_bnrelu,cbr512_16x16,cbr512 VERBOSE=1 $G"
