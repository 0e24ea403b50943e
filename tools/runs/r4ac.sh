#!/bin/bash
# conv1 forward NT vs xl, checkpoint test on tamed residual branches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "200|r4ac_ab2048|python -u tools/fold_dgrad_ab.py --batch 2048 > gpurun_out/r4ac_ab2048.md" \
  "150|r4ac_ab256|python -u tools/fold_dgrad_ab.py --batch 256 > gpurun_out/r4ac_ab256.md" \
  "250|r4ac_ckpt|DMP_RUN_UNVALIDATED=1 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_checkpointing.py -rA"
