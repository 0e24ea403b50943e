set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests/test_gpu_convergence.py tests/test_gpu_ddp.py tests/test_gpu_depthwise.py tests/test_gpu_gemm.py tests/test_gpu_gemm_tn.py tests/test_gpu_gemm_tn_xl.py tests/test_gpu_gemm_x2.py tests/test_gpu_gemm_xl.py tests/test_gpu_gemm_xl_bm.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_gemm_xl_tail.py tests/test_gpu_graph.py tests/test_gpu_kernels.py tests/test_gpu_layernorm.py tests/test_gpu_linear.py tests/test_gpu_loss.py tests/test_gpu_models.py tests/test_gpu_parity_train.py tests/test_gpu_pipeline.py tests/test_gpu_pool.py tests/test_gpu_stem.py tests/test_gpu_vit_xl.py tests/test_gpu_wgrad3x3.py tests/test_gpu_wgrad_stream.py  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_suite2.log 2>&1 || { tail -40 gpurun_out/gpu_suite2.log; exit 1; }
tail -3 gpurun_out/gpu_suite2.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
