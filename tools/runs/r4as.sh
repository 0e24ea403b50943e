#!/bin/bash
# final build: default GPU suite as the driver runs it, smoke, headline bench, ViT, MobileNetV2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "800|r4as_suite|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "200|r4as_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|r4as_b2048|python bench.py" \
  "150|r4as_vit|python bench.py --model vit_b_16 --steps 20 --warmup 5" \
  "150|r4as_mnv2|python bench.py --model mobilenetv2 --steps 30 --warmup 5"
