#!/bin/bash
# graph replay bisect on layer4 (two blocks) by feature
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "60|r4j_l4|ONLY=layer4,layer3[0] $G" \
  "60|r4j_fuse|ONLY=layer4 DMP_DISABLE=fuse_bn_bwd $G" \
  "60|r4j_compact|ONLY=layer4 DMP_DISABLE=compact_shortcut $G" \
  "60|r4j_xl|ONLY=layer4 DMP_DISABLE=xl_conv $G" \
  "60|r4j_igemm|ONLY=layer4 DMP_DISABLE=igemm $G" \
  "60|r4j_all|ONLY=layer4 DMP_DISABLE=fuse_bn_bwd,compact_shortcut,xl_conv3,xl_conv,igemm $G"
