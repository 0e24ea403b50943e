#!/bin/bash
# x2 with the two-stage ring vs xl; LayerNorm prefetch; NT conv epilogues; ViT plain-GEMM A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
B="python bench.py --batch-size 256 --steps 30 --warmup 10"
B2="python bench.py --steps 15 --warmup 5"
bash tools/gpu_steps.sh \
  "200|r4s_tests|$P tests/test_gpu_gemm_x2.py tests/test_gpu_layernorm.py tests/test_gpu_gemm_xl_conv.py" \
  "200|r4s_x2_bench|python -u tools/x2_bench.py > gpurun_out/r4s_x2_bench.md" \
  "200|r4s_x2_bench2048|python -u tools/x2_bench.py --batch 2048 > gpurun_out/r4s_x2_bench2048.md" \
  "100|r4s_nt0a|$B" "100|r4s_nt1a|DMP_XL_NT=1 $B" "100|r4s_nt0b|$B" "100|r4s_nt1b|DMP_XL_NT=1 $B" \
  "150|r4s_nt0c|$B2" "150|r4s_nt1c|DMP_XL_NT=1 $B2" && \
bash tools/runs/r4r.sh
