#!/bin/bash
# fold GEMMs via hipBLASLt, attention VALU cleanup + 2-tile forward, DP graph diagnosis
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PYTHONUNBUFFERED=1 DMP_RUN_UNVALIDATED=1
P="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_MFMA"
bash tools/gpu_steps.sh \
  "200|r4e_fold_tests|$P tests/test_gpu_bn_fold.py -k 'coefficient or ds_kernels'" \
  "200|r4e_b256|python bench.py --batch-size 256 --steps 30 --warmup 10" \
  "240|r4e_attn_tests|$P tests/test_gpu_attention.py" \
  "150|r4e_attn_bench|B=256 python -u tools/attn_bench.py" \
  "150|r4e_dpdiag|python -u tools/dp_graph_diag.py" \
  "240|r4e_b2048|python bench.py --steps 20 --warmup 5" \
  "90|r4e_pmc1_v0|B=256 VARIANT=0,0 ITERS=3 rocprofv3 --pmc $C1 -d gpurun_out/r4e_pmc1_v0 -o p --output-format csv -- python3 tools/attn_bench.py" \
  "90|r4e_pmc2_v0|B=256 VARIANT=0,0 ITERS=3 rocprofv3 --pmc $C2 -d gpurun_out/r4e_pmc2_v0 -o p --output-format csv -- python3 tools/attn_bench.py" \
  "90|r4e_pmc1_v3|B=256 VARIANT=3,1 ITERS=3 rocprofv3 --pmc $C1 -d gpurun_out/r4e_pmc1_v3 -o p --output-format csv -- python3 tools/attn_bench.py" \
  "90|r4e_pmc2_v3|B=256 VARIANT=3,1 ITERS=3 rocprofv3 --pmc $C2 -d gpurun_out/r4e_pmc2_v3 -o p --output-format csv -- python3 tools/attn_bench.py"
