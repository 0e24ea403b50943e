set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_depthwise.py tests/test_gpu_kernels.py tests/test_gpu_bn_bwd_fused.py tests/test_gpu_bn_fold.py tests/test_gpu_layernorm.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dw.log 2>&1 || { tail -40 gpurun_out/t_dw.log; exit 1; }
tail -2 gpurun_out/t_dw.log
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
for r in head new head2 new2; do
  case $r in head*) export DMP_NATIVE_SO=$PWD/ab_so/_C_head.so;; *) unset DMP_NATIVE_SO;; esac
  timeout -k 10 200 python bench.py --model mobilenetv2 --steps 30 --warmup 10 > gpurun_out/dw_mnv2_$r.json 2>gpurun_out/dw_mnv2_$r.err || exit 1
  timeout -k 10 200 python bench.py > gpurun_out/dw_r50_$r.json 2>gpurun_out/dw_r50_$r.err || exit 1
  timeout -k 10 200 python bench.py --model vit_b_16 --steps 30 --warmup 10 > gpurun_out/dw_vit_$r.json 2>gpurun_out/dw_vit_$r.err || exit 1
  echo "$r mnv2 $(js gpurun_out/dw_mnv2_$r.json) | r50 $(js gpurun_out/dw_r50_$r.json) | vit $(js gpurun_out/dw_vit_$r.json)"
done
unset DMP_NATIVE_SO
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnv2 -o run -- python3 bench.py --model mobilenetv2 --steps 8 --warmup 3 > gpurun_out/prof_mnv2.log 2>&1 || exit 1
echo done
