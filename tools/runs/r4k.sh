#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "60|r4k_verbose|ONLY=layer4 VERBOSE=1 $G" \
  "60|r4k_noupd|ONLY=layer4 NOUPDATE=1 $G" \
  "60|r4k_noupd_samex|ONLY=layer4 NOUPDATE=1 SAMEX=1 VERBOSE=1 $G"
