set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_loss.py tests/test_gpu_grad_accum.py tests/test_gpu_pipeline.py > gpurun_out/ga.log 2>&1 &&
timeout -k 10 120 python -u tools/graph_branch_probe.py > gpurun_out/branch.log 2>&1 &&
timeout -k 10 200 python -u bench.py --parallel pipe --model mobilenetv2 --steps 10 --warmup 3 > gpurun_out/pipe_bench.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r50_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe_r6b -o run -- python -u bench.py --parallel pipe --model mobilenetv2 --steps 4 --warmup 3 > gpurun_out/pipe_prof.log 2>&1
