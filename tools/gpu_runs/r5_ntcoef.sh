set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bn_fold.py tests/test_gpu_gemm_xl_conv.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_nt.log 2>&1 || { tail -40 gpurun_out/t_nt.log; exit 1; }
tail -2 gpurun_out/t_nt.log
DMP_NATIVE_SO=$PWD/ab_so/_C_ntb.so timeout -k 10 500 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_bn_fold.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ntb.log 2>&1 || { tail -40 gpurun_out/t_ntb.log; exit 1; }
tail -2 gpurun_out/t_ntb.log
for r in head a b head2 a2 b2; do
  case $r in head*) export DMP_NATIVE_SO=$PWD/ab_so/_C_head.so;; b*) export DMP_NATIVE_SO=$PWD/ab_so/_C_ntb.so;; *) unset DMP_NATIVE_SO;; esac
  timeout -k 10 200 python bench.py > gpurun_out/nt_$r.json 2>gpurun_out/nt_$r.err || exit 1
  timeout -k 10 200 python bench.py --batch-size 256 --steps 30 --warmup 10 > gpurun_out/nt256_$r.json 2>gpurun_out/nt256_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/nt_$r.json) | bs256 $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/nt256_$r.json)"
done
