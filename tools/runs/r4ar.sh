#!/bin/bash
# convergence 224 twice with curves after the NT BN-backward variants
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T="python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py -k 224"
bash tools/gpu_steps.sh "200|r4ar_c1|DMP_CONVERGENCE_OUT=gpurun_out/conv_r4ar1.json $T" "200|r4ar_c2|DMP_CONVERGENCE_OUT=gpurun_out/conv_r4ar2.json $T"
