#!/bin/bash
# PMC passes over the halo wgrad kernel (one counter set per run)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3pmc; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d $O/p1 -o p1 --output-format csv -- python3 tools/wgrad_bench.py --only ${1:-256} --loop 3 > $O/p1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_MFMA -d $O/p2 -o p2 --output-format csv -- python3 tools/wgrad_bench.py --only ${1:-256} --loop 3 > $O/p2.log 2>&1 || exit $?
echo pmc-done
