#!/bin/bash
# final-state default GPU suite, smoke(), and the README benchmark rows
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "800|r4ag_suite|python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests" \
  "200|r4ag_smoke|python -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "150|r4ag_b2048|python bench.py" \
  "150|r4ag_b256|python bench.py --batch-size 256 --steps 30 --warmup 5" \
  "150|r4ag_vit|python bench.py --model vit_b_16 --steps 20 --warmup 5" \
  "150|r4ag_mnv2|python bench.py --model mobilenetv2 --steps 30 --warmup 5"
