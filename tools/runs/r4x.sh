#!/bin/bash
# gemm_nt transposed-accumulator staging: numerics, step roofline at bs2048, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "500|r4x_tests|$P tests/test_gpu_gemm.py tests/test_gpu_conv_igemm.py tests/test_gpu_bn_bwd_fused.py tests/test_gpu_bn_fold.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_linear.py tests/test_gpu_models.py tests/test_gpu_conv_halo.py tests/test_gpu_stem.py" \
  "300|r4x_roof|python -u tools/step_roofline.py > gpurun_out/r4x_roof2048.md" \
  "150|r4x_b2048|python bench.py --steps 20 --warmup 5" \
  "150|r4x_b256|python bench.py --batch-size 256 --steps 30 --warmup 5"
