#!/bin/bash
# DP graphs multi-step diagnosis (streams on / off), checkpointing test vs same-kernel reference
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "150|r4g_diag_streams|python -u tools/dp_graph_diag.py --steps 3 --lr 0.05" \
  "150|r4g_diag_nostreams|DMP_DP_GRAPH_STREAMS=0 python -u tools/dp_graph_diag.py --steps 3 --lr 0.05" \
  "150|r4g_diag_lr01|python -u tools/dp_graph_diag.py --steps 3 --lr 0.01 --batch 64" \
  "300|r4g_ckpt|$P tests/test_gpu_checkpointing.py" \
  "300|r4g_fold_head|$P tests/test_gpu_bn_fold.py -k headline"
