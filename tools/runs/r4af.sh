#!/bin/bash
# A/B after the epilogue changes: ViT plain GEMMs lib vs xl; fold products hipBLASLt vs tiled at bs2048
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
V="python bench.py --model vit_b_16 --batch-size 256 --steps 20 --warmup 5"
R="python bench.py --steps 15 --warmup 5"
bash tools/gpu_steps.sh \
  "150|r4af_vit_lib|DMP_LINEAR_PLAIN=lib $V" \
  "150|r4af_vit_xl|DMP_LINEAR_PLAIN=xl $V" \
  "150|r4af_vit_lib2|DMP_LINEAR_PLAIN=lib $V" \
  "150|r4af_vit_xl2|DMP_LINEAR_PLAIN=xl $V" \
  "150|r4af_r50_f1|DMP_FOLD_GEMM=1 $R" \
  "150|r4af_r50_f2|DMP_FOLD_GEMM=2 $R" \
  "150|r4af_r50_f1b|DMP_FOLD_GEMM=1 $R" \
  "150|r4af_r50_f2b|DMP_FOLD_GEMM=2 $R"
