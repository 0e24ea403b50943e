#!/bin/bash
# transposed-accumulator staging + pointer-increment epilogue in gemm_xl PIPE 7/8: numerics, xl timings, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "400|r4w_tests|$P tests/test_gpu_gemm_xl.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_conv_xl.py tests/test_gpu_vit_xl.py tests/test_gpu_linear.py tests/test_gpu_bn_fold.py tests/test_gpu_gemm_x2.py" \
  "200|r4w_x2_2048|python -u tools/x2_bench.py --batch 2048 > gpurun_out/r4w_x2_2048.md" \
  "150|r4w_x2_256|python -u tools/x2_bench.py --batch 256 > gpurun_out/r4w_x2_256.md" \
  "150|r4w_b2048|python bench.py --steps 20 --warmup 5" \
  "150|r4w_b256|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "200|r4w_gap|python -u tools/conv_xl_gap.py --batch 2048 > gpurun_out/r4w_gap.md" \
  "150|r4w_vit|python bench.py --model vit_b_16 --batch-size 256 --steps 20 --warmup 5"
