set -o pipefail
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm_tn_xl.py tests/test_gpu_bn_fold.py tests/test_gpu_models.py > gpurun_out/strided.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r50_a.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch-size 256 --steps 10 --warmup 3 > gpurun_out/r50_256a.log 2>&1
