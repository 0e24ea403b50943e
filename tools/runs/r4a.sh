set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_xl.py tests/test_gpu_gemm_tn_xl.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_vit_xl.py tests/test_gpu_attention.py > gpurun_out/r4a_tests.log 2>&1 && \
timeout -k 10 120 env B=256 python -u tools/attn_bench.py > gpurun_out/r4a_attn.log 2>&1 && \
timeout -k 10 400 python -u tools/ring_bench.py --rounds 5 --iters 10 > gpurun_out/r4a_ring.log 2>&1
