#!/bin/bash
# graph replay bisect by module; fold mode A/B at bs256 (interleaved), bs256 trace
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
B="python bench.py --batch-size 256 --steps 30 --warmup 10"
bash tools/gpu_steps.sh \
  "200|r4i_bisect|python -u tools/graph_replay_bisect.py" \
  "100|r4i_f2a|DMP_FOLD_GEMM=2 $B" \
  "100|r4i_f1a|DMP_FOLD_GEMM=1 $B" \
  "100|r4i_f0a|DMP_FOLD_GEMM=0 $B" \
  "100|r4i_f2b|DMP_FOLD_GEMM=2 $B" \
  "100|r4i_f1b|DMP_FOLD_GEMM=1 $B" \
  "100|r4i_f0b|DMP_FOLD_GEMM=0 $B" \
  "300|r4i_prof256|rocprofv3 --kernel-trace --stats -d gpurun_out/r4i_prof256 -o prof --output-format csv -- python3 bench.py --batch-size 256 --steps 12 --warmup 8"
