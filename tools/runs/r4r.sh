#!/bin/bash
# ViT-B/16: plain GEMMs (qkv fwd, data gradients) and weight gradients on gemm_xl vs hipBLASLt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
V="python bench.py --model vit_b_16 --batch-size 256 --steps 10 --warmup 5"
bash tools/gpu_steps.sh \
  "120|r4r_xl_a|$V" \
  "120|r4r_lib_a|DMP_LINEAR_PLAIN=lib $V" \
  "120|r4r_libtn_a|DMP_LINEAR_PLAIN=lib DMP_DISABLE=tn_xl $V" \
  "120|r4r_xl_b|$V" \
  "120|r4r_lib_b|DMP_LINEAR_PLAIN=lib $V" \
  "120|r4r_libtn_b|DMP_LINEAR_PLAIN=lib DMP_DISABLE=tn_xl $V"
