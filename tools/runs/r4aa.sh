#!/bin/bash
# fold dgrad / forward NT vs xl A/B at bs2048 and bs256; checkpoint test with the fp32 oracle
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "200|r4aa_fold2048|python -u tools/fold_dgrad_ab.py --batch 2048 > gpurun_out/r4aa_fold2048.md" \
  "150|r4aa_fold256|python -u tools/fold_dgrad_ab.py --batch 256 > gpurun_out/r4aa_fold256.md" \
  "250|r4aa_ckpt|DMP_RUN_UNVALIDATED=1 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_checkpointing.py -rA"
