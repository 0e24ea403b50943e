#!/bin/bash
# PMC of the BN-backward conv epilogue GEMM on the final build (planning data for the next round)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P4="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES"
for cfg in "l2_conv3 bnbwd_res" "l3_conv3 bnbwd" "l3_conv3 moments"; do
  set -- $cfg
  for pass in "p1:$P1" "p4:$P4" "p2:FETCH_SIZE" "p3:WRITE_SIZE"; do
    nm=${pass%%:*}; ctr=${pass#*:}
    timeout -s KILL 60 env SHAPE=$1 MODE=$2 rocprofv3 --pmc $ctr -d gpurun_out/r4ao_pmc_${1}_${2}_$nm -o p --output-format csv -- python3 tools/gemm_pmc_probe.py > gpurun_out/r4ao_pmc_${1}_${2}_$nm.log 2>&1 || exit $?
  done
done
echo pmc-done
