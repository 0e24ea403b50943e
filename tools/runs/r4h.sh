#!/bin/bash
# graph-replay bisect; fold tiled kernel tests + bs256 A/B (fold modes, fold off, graph)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
G="python -u tools/graph_replay_check.py --steps 3"
bash tools/gpu_steps.sh \
  "120|r4h_gr_all|$G" \
  "120|r4h_gr_noxl3|DMP_DISABLE=xl_conv3 $G" \
  "120|r4h_gr_nofuse|DMP_DISABLE=fuse_bn_bwd $G" \
  "120|r4h_gr_noigemm|DMP_DISABLE=igemm $G" \
  "120|r4h_gr_r50|$G --arch resnet50 --batch 8" \
  "200|r4h_fold_tests|$P tests/test_gpu_bn_fold.py -k 'coefficient or ds_kernels or headline'" \
  "120|r4h_b256|python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "120|r4h_b256_nofold|DMP_DISABLE=bn_fold python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "120|r4h_b256_graph|python bench.py --batch-size 256 --steps 30 --warmup 10 --graph" \
  "200|r4h_b2048|python bench.py --steps 20 --warmup 5"
