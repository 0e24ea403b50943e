set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_pipeline.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_pq.log 2>&1 || { tail -30 gpurun_out/t_pq.log; exit 1; }
tail -2 gpurun_out/t_pq.log
timeout -k 10 120 python tools/pool_bn_bench.py > gpurun_out/pq_new.md 2>&1 || exit 1
DMP_POOL_BWD1=1 timeout -k 10 120 python tools/pool_bn_bench.py > gpurun_out/pq_old.md 2>&1 || exit 1
echo quad; cat gpurun_out/pq_new.md; echo one-pixel; cat gpurun_out/pq_old.md
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
for r in a b a2 b2; do
  case $r in b*) export DMP_POOL_BWD1=1;; *) unset DMP_POOL_BWD1;; esac
  timeout -k 10 200 python bench.py > gpurun_out/pq_r50_$r.json 2>gpurun_out/pq_r50_$r.err || exit 1
  echo "$r r50 $(js gpurun_out/pq_r50_$r.json)"
done
unset DMP_POOL_BWD1
timeout -k 10 300 python tools/torch_op_sources.py --model mobilenetv2 --batch-size 512 --steps 3 > gpurun_out/mnv2_src.md 2>gpurun_out/mnv2_src.err || { tail -20 gpurun_out/mnv2_src.err; exit 1; }
head -30 gpurun_out/mnv2_src.md
