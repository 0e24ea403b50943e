set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_convergence.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pg.log 2>&1 || { tail -30 gpurun_out/t_pg.log; exit 1; }
tail -2 gpurun_out/t_pg.log
timeout -k 10 300 python tools/torch_op_sources.py --model mobilenetv2 --batch-size 512 --steps 3 > gpurun_out/mnv2_src.md 2>gpurun_out/mnv2_src.err || { tail -20 gpurun_out/mnv2_src.err; exit 1; }
cat gpurun_out/mnv2_src.md
