set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fold2 -o run -- python -u tools/fold_gemm_ab.py --batch 256 --steps 5 --rounds 1 --modes 2 > gpurun_out/fold_tr2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fold1 -o run -- python -u tools/fold_gemm_ab.py --batch 256 --steps 5 --rounds 1 --modes 1 > gpurun_out/fold_tr1.log 2>&1
