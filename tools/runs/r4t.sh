#!/bin/bash
# TN weight gradients incl. hipBLASLt; ViT with plain GEMMs on the library (tests + bench)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "200|r4t_tests|$P tests/test_gpu_vit_xl.py tests/test_gpu_layernorm.py" \
  "200|r4t_tn256|python -u tools/tn256_bench.py > gpurun_out/r4t_tn256.md" \
  "300|r4t_tn2048|python -u tools/tn256_bench.py --batch 2048 > gpurun_out/r4t_tn2048.md" \
  "150|r4t_vit|python bench.py --model vit_b_16 --batch-size 256 --steps 20 --warmup 5"
