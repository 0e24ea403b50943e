#!/bin/bash
# final-build kernel traces: ResNet-50 batch 256 and ViT-B/16
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "300|r4an_prof256|rocprofv3 --kernel-trace --stats -d gpurun_out/r4an_prof256 -o prof --output-format csv -- python3 bench.py --batch-size 256 --steps 12 --warmup 8" \
  "300|r4an_profvit|rocprofv3 --kernel-trace --stats -d gpurun_out/r4an_profvit -o prof --output-format csv -- python3 bench.py --model vit_b_16 --steps 8 --warmup 5"
