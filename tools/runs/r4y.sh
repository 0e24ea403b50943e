#!/bin/bash
# full default GPU suite after the epilogue staging changes, then the two still-unvalidated tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "900|r4y_suite|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "250|r4y_unval|DMP_RUN_UNVALIDATED=1 DMP_CONVERGENCE_OUT=gpurun_out/conv_r4y.json python -u -m pytest -q --timeout 300 --timeout-method thread -m 'gpu and unvalidated' tests -rA"
