#!/bin/bash
# stability of the chaotic-numerics tests: three runs each of the checkpoint and DDP ordering tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_checkpointing.py tests/test_gpu_ddp.py -k 'checkpointed or ordering' -rA"
bash tools/gpu_steps.sh "300|r4ai_1|$T" "300|r4ai_2|$T" "300|r4ai_3|$T"
