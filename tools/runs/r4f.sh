#!/bin/bash
# defaults changed (attention 2/0, x2 rule, fold BLAS), bs256 trace, TN at bs256, DP graphs on streams
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "240|r4f_quick_tests|$P tests/test_gpu_gemm_x2.py tests/test_gpu_attention.py tests/test_gpu_vit_xl.py" \
  "200|r4f_b256|python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "300|r4f_prof256|rocprofv3 --kernel-trace --stats -d gpurun_out/r4f_prof256 -o prof --output-format csv -- python3 bench.py --batch-size 256 --steps 12 --warmup 8" \
  "200|r4f_tn256|python -u tools/tn256_bench.py > gpurun_out/r4f_tn256.md" \
  "300|r4f_dp_tests|$P tests/test_data_parallel.py -m gpu" \
  "200|r4f_dp4_graphs|python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --dp-graphs" \
  "300|r4f_ckpt_fold|$P tests/test_gpu_checkpointing.py tests/test_gpu_bn_fold.py" \
  "200|r4f_vit|python bench.py --model vit_b_16 --batch-size 256 --steps 10 --warmup 5" \
  "450|r4f_conv224|DMP_CONVERGENCE_OUT=gpurun_out/r4f_conv.json $P --timeout 420 tests/test_gpu_convergence.py -k 224"
