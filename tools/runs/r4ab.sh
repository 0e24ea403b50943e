#!/bin/bash
# folded dgrad on the ping-pong GEMM from cin >= 128: numerics, benches, bs2048 kernel trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "400|r4ab_tests|DMP_RUN_UNVALIDATED=1 $P tests/test_gpu_gemm_x2.py tests/test_gpu_bn_fold.py tests/test_gpu_checkpointing.py tests/test_gpu_models.py" \
  "150|r4ab_b2048|python bench.py --steps 20 --warmup 5" \
  "150|r4ab_b256|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "300|r4ab_prof2048|rocprofv3 --kernel-trace --stats -d gpurun_out/r4ab_prof2048 -o prof --output-format csv -- python3 bench.py --steps 6 --warmup 4"
