#!/bin/bash
# checkpoint-test diagnosis (fused / checkpointed / fp32 oracle gradients), then the default GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "200|r4z_diag8|python -u tools/ckpt_grad_diag.py --batch 8 --size 64 --seeds 3" \
  "200|r4z_diag32|python -u tools/ckpt_grad_diag.py --batch 32 --size 64 --seeds 2" \
  "750|r4z_suite|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests"
