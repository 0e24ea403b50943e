#!/bin/bash
# MIOpen left out of captured graphs; l4 s2 wgrad on conv_wgrad_xl; graph / DP re-checks
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
G="python -u tools/graph_replay_bisect.py"
bash tools/gpu_steps.sh \
  "150|r4o_wgs2|python -u tools/wgrad_s2_bench.py" \
  "120|r4o_bisect|ONLY=conv_only,cbr512,layer4,layer3,whole $G" \
  "150|r4o_diag|python -u tools/dp_graph_diag.py --steps 3 --lr 0.05" \
  "150|r4o_diag_gen|DMP_GENERIC_BWD=1 python -u tools/dp_graph_diag.py --steps 3 --lr 0.05" \
  "300|r4o_conv_tests|$P tests/test_gpu_conv_igemm.py tests/test_gpu_gemm_tn_xl.py" \
  "300|r4o_dp_tests|$P tests/test_data_parallel.py -m gpu" \
  "200|r4o_b2048|python bench.py --steps 20 --warmup 5" \
  "200|r4o_b256|python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "200|r4o_b256_graph|python bench.py --batch-size 256 --steps 30 --warmup 10 --graph" \
  "200|r4o_dp4_graphs|python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --dp-graphs"
