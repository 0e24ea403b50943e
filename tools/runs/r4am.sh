#!/bin/bash
# final build: default GPU suite (as the driver runs it), smoke, headline bench x2, batch 256, ViT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "800|r4am_suite|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "200|r4am_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|r4am_b2048|python bench.py" \
  "150|r4am_b2048b|python bench.py" \
  "150|r4am_b256|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "150|r4am_vit|python bench.py --model vit_b_16 --steps 20 --warmup 5"
