set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm_xl.py tests/test_gpu_gemm_xl_conv.py tests/test_gpu_conv_xl.py tests/test_gpu_gemm_xl_bm.py tests/test_gpu_gemm_xl_tail.py tests/test_gpu_vit_xl.py tests/test_gpu_bn_fold.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_epi.log 2>&1 || { tail -40 gpurun_out/t_epi.log; exit 1; }
tail -2 gpurun_out/t_epi.log
timeout -k 10 300 python tools/xl_phase_trace.py > gpurun_out/xl_phase2.md 2>&1 || { cat gpurun_out/xl_phase2.md; exit 1; }
cat gpurun_out/xl_phase2.md
for r in e1 e2 e3; do
  timeout -k 10 200 python bench.py > gpurun_out/epi_$r.json 2>gpurun_out/epi_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/epi_$r.json)"
done
timeout -k 10 200 python bench.py --model vit_b_16 --batch-size 256 --steps 10 --warmup 5 > gpurun_out/epi_vit.json 2>gpurun_out/epi_vit.err || exit 1
echo "vit $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/epi_vit.json)"
