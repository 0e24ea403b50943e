#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "60|r4l_ref|ONLY=layer4 REFMODE=1 $G" \
  "60|r4l_zero|ONLY=layer4 ZERO_GRADS=1 VERBOSE=1 $G"
