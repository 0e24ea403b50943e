#!/bin/bash
# layer-3 conv1 forward on the ping-pong GEMM: tests, benches; VALU / LDS PMC of the conv epilogues after the staging change
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
bash tools/gpu_steps.sh \
  "300|r4ad_tests|$P tests/test_gpu_models.py tests/test_gpu_bn_bwd_fused.py tests/test_gpu_bn_fold.py tests/test_gpu_gemm_xl_conv.py" \
  "150|r4ad_b2048|python bench.py --steps 20 --warmup 5" \
  "150|r4ad_b256|python bench.py --batch-size 256 --steps 30 --warmup 5" || exit $?
P4="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES"
for cfg in "l2_conv3 affine_res" "l3_conv3 affine" "l3_conv3 bnbwd"; do
  set -- $cfg
  timeout -s KILL 60 env SHAPE=$1 MODE=$2 rocprofv3 --pmc $P4 -d gpurun_out/r4ad_pmc_${1}_${2} -o p --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/r4ad_pmc_${1}_${2}.log 2>&1 || exit $?
done
echo pmc-done
