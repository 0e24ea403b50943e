#!/bin/bash
# LayerNorm two rows per wave at D = 768: numerics, ViT bench and roofline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "300|r4ae_tests|$P tests/test_gpu_layernorm.py tests/test_gpu_vit_xl.py tests/test_gpu_models.py" \
  "150|r4ae_vit|python bench.py --model vit_b_16 --batch-size 256 --steps 20 --warmup 5" \
  "300|r4ae_vitroof|python -u tools/step_roofline.py --model vit_b_16 --batch-size 256 > gpurun_out/r4ae_vitroof.md" \
  "150|r4ae_vit2|python bench.py --model vit_b_16 --batch-size 256 --steps 20 --warmup 5"
