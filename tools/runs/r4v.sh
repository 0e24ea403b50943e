#!/bin/bash
# convergence 224 (default routes x2, eager conv_wgrad_xl off x1) with curves; tn_xl row threshold A/B at bs2048
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
T="DMP_RUN_UNVALIDATED=1 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_convergence.py -k 224"
bash tools/gpu_steps.sh \
  "200|r4v_conv_a|DMP_CONVERGENCE_OUT=gpurun_out/conv_a.json $T" \
  "200|r4v_conv_b|DMP_CONVERGENCE_OUT=gpurun_out/conv_b.json $T" \
  "200|r4v_conv_nowg|DMP_XL_WGRAD_MAX_ROWS=0 DMP_CONVERGENCE_OUT=gpurun_out/conv_nowg.json $T" \
  "150|r4v_b2048_100k|python bench.py --steps 20 --warmup 5" \
  "150|r4v_b2048_150k|DMP_TN_XL_MIN_ROWS=150000 python bench.py --steps 20 --warmup 5" \
  "150|r4v_b2048_100k_2|python bench.py --steps 20 --warmup 5" \
  "150|r4v_b2048_150k_2|DMP_TN_XL_MIN_ROWS=150000 python bench.py --steps 20 --warmup 5" \
  "150|r4v_b256_graph|python bench.py --batch-size 256 --graph --steps 30 --warmup 5"
