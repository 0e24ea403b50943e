#!/bin/bash
# full default GPU suite (as the driver runs it), then the unvalidated tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "900|r4p_suite|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "600|r4p_unval|DMP_RUN_UNVALIDATED=1 python -u -m pytest tests -m 'gpu and unvalidated' -q --timeout 420 --timeout-method thread"
