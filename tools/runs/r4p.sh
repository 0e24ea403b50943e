#!/bin/bash
# full default GPU suite (as the driver runs it), then the unvalidated tests
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
bash tools/gpu_steps.sh \
  "900|r4p_suite|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "600|r4p_unval|DMP_RUN_UNVALIDATED=1 python -u -m pytest tests -m 'gpu and unvalidated' -q --timeout 420 --timeout-method thread"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P4="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES"
for cfg in "l2_conv3 affine_res" "l3_conv3 affine" "l3_conv3 bnbwd"; do
  set -- $cfg
  for pass in "p1:$P1" "p2:FETCH_SIZE" "p3:WRITE_SIZE" "p4:$P4"; do
    nm=${pass%%:*}; ctr=${pass#*:}
    timeout -s KILL 60 env SHAPE=$1 MODE=$2 rocprofv3 --pmc $ctr -d gpurun_out/r4p_pmc_${1}_${2}_$nm -o p --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/r4p_pmc_${1}_${2}_$nm.log 2>&1 || exit $?
  done
done
echo pmc-done
