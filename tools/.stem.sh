set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stem.py tests/test_gpu_bn_bwd_fused.py tests/test_gpu_models.py tests/test_gpu_bn_fold.py tests/test_gpu_kernels.py > gpurun_out/stem_t.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_stem -o run -- python -u bench.py --batch-size 256 --steps 5 --warmup 3 > gpurun_out/stem_tr.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch-size 256 --steps 20 --warmup 3 > gpurun_out/r50_256b.log 2>&1 &&
timeout -k 10 300 python -u bench.py --parallel pipe --model mobilenetv2 --steps 10 --warmup 3 > gpurun_out/pipe_b.log 2>&1
