#!/bin/bash
# tn_xl 100k-row threshold on the headline benches; MobileNetV2; unvalidated tests; default GPU suite
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "200|r4u_bs2048|python bench.py --steps 20 --warmup 5" \
  "150|r4u_bs256|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "150|r4u_mnv2|python bench.py --model mobilenetv2 --steps 30 --warmup 5" \
  "150|r4u_mnv2_pipe|python bench.py --parallel pipe --model mobilenetv2 --steps 30 --warmup 5" \
  "480|r4u_unval|DMP_RUN_UNVALIDATED=1 python -u -m pytest -q --timeout 300 --timeout-method thread -m 'gpu and unvalidated' tests -rA"
