#!/bin/bash
# round 4 collection run: every pending measurement in one box session
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "200|r4d_attn_tests|$P tests/test_gpu_attention.py" \
  "120|r4d_attn_bench|B=256 python -u tools/attn_bench.py" \
  "300|r4d_roof_r50|python -u tools/step_roofline.py > gpurun_out/r4d_roof_r50.md" \
  "300|r4d_roof_r50_256|python -u tools/step_roofline.py --batch-size 256 > gpurun_out/r4d_roof_r50_256.md" \
  "300|r4d_roof_vit|python -u tools/step_roofline.py --model vit_b_16 > gpurun_out/r4d_roof_vit.md" \
  "200|r4d_b256|python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "300|r4d_prof256|rocprofv3 --kernel-trace --stats -d gpurun_out/r4d_prof256 -o prof --output-format csv -- python3 bench.py --batch-size 256 --steps 6 --warmup 3" \
  "400|r4d_dp_tests|$P tests/test_data_parallel.py tests/test_gpu_checkpointing.py tests/test_gpu_bn_fold.py -m gpu" \
  "200|r4d_dp4_eager|python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --phase-times" \
  "200|r4d_dp4_graphs|python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --dp-graphs" \
  "400|r4d_conv224|DMP_CONVERGENCE_OUT=gpurun_out/r4d_conv.json $P --timeout 380 tests/test_gpu_convergence.py -k 224" || exit $?
bash tools/gpu_steps.sh \
  "200|r4d_x2_tests|$P tests/test_gpu_gemm_x2.py" \
  "200|r4d_x2_bench|python -u tools/x2_bench.py > gpurun_out/r4d_x2_bench.md"
