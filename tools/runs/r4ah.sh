#!/bin/bash
# default GPU suite on the final state (no -x: the full picture), then its summary
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "900|r4ah_suite|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests -rf"
