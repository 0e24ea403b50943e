#!/bin/bash
# split-K tail of the ping-pong GEMMs: numerics (new + every GEMM/conv test), tail probe, benches
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "400|r4ak_tests|$P tests/test_gpu_gemm_xl_tail.py tests/test_gpu_conv_xl.py tests/test_gpu_gemm_xl.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_gemm_x2.py tests/test_gpu_bn_fold.py tests/test_gpu_models.py tests/test_gpu_vit_xl.py tests/test_gpu_linear.py" \
  "200|r4ak_tail_on|python -u tools/tile_tail_probe.py > gpurun_out/r4ak_tail_on.md" \
  "200|r4ak_tail_off|DMP_XL_TAIL=0 python -u tools/tile_tail_probe.py > gpurun_out/r4ak_tail_off.md" \
  "150|r4ak_b2048_on|python bench.py --steps 20 --warmup 5" \
  "150|r4ak_b2048_off|DMP_XL_TAIL=0 python bench.py --steps 20 --warmup 5" \
  "150|r4ak_b256_on|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "150|r4ak_b256_off|DMP_XL_TAIL=0 python bench.py --batch-size 256 --steps 30 --warmup 5"
