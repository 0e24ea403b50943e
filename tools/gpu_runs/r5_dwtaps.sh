set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_depthwise.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dwt.log 2>&1 || { tail -40 gpurun_out/t_dwt.log; exit 1; }
tail -2 gpurun_out/t_dwt.log
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
for r in head new head2 new2 head3 new3; do
  case $r in head*) export DMP_NATIVE_SO=$PWD/ab_so/_C_head.so;; *) unset DMP_NATIVE_SO;; esac
  timeout -k 10 200 python bench.py --model mobilenetv2 --steps 40 --warmup 10 > gpurun_out/dwt_mnv2_$r.json 2>gpurun_out/dwt_mnv2_$r.err || exit 1
  echo "$r mnv2 $(js gpurun_out/dwt_mnv2_$r.json)"
done
unset DMP_NATIVE_SO
timeout -k 10 300 python tools/torch_op_sources.py --model mobilenetv2 --batch-size 512 --steps 3 > gpurun_out/mnv2_src2.md 2>gpurun_out/mnv2_src2.err || { tail -20 gpurun_out/mnv2_src2.err; exit 1; }
grep "^|" gpurun_out/mnv2_src2.md | head -14
