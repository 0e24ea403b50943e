set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_bn_fold.py > gpurun_out/fold_t.log 2>&1 &&
timeout -k 10 300 python -u tools/fold_gemm_ab.py --batch 256 --steps 20 --rounds 3 > gpurun_out/fold_ab256.log 2>&1 &&
timeout -k 10 300 python -u tools/fold_gemm_ab.py --batch 2048 --steps 5 --rounds 3 > gpurun_out/fold_ab2048.log 2>&1
