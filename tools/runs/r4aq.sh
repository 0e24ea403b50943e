#!/bin/bash
# NT conv GEMM BN-backward variants: numerics, roofline, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "500|r4aq_tests|$P tests/test_gpu_gemm.py tests/test_gpu_bn_bwd_fused.py tests/test_gpu_bn_fold.py tests/test_gpu_conv_igemm.py tests/test_gpu_gemm_x2.py tests/test_gpu_models.py tests/test_gpu_convergence.py tests/test_gpu_ddp.py" \
  "300|r4aq_roof|python -u tools/step_roofline.py > gpurun_out/r4aq_roof2048.md" \
  "150|r4aq_b2048|python bench.py" \
  "150|r4aq_b256|python bench.py --batch-size 256 --steps 30 --warmup 5"
