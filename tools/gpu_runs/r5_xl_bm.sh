set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_xl_bm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_bm.log 2>&1 || { tail -30 gpurun_out/t_bm.log; exit 1; }
tail -3 gpurun_out/t_bm.log
timeout -k 10 300 python tools/xl_bm_bench.py > gpurun_out/xl_bm_bench.md 2>&1 || exit 1
cat gpurun_out/xl_bm_bench.md
for r in a1 b1 a2 b2; do
  if [[ $r == a* ]]; then export DMP_XL_BM=0; else export DMP_XL_BM=-1; fi
  timeout -k 10 200 python bench.py > gpurun_out/bm_$r.json 2>gpurun_out/bm_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/bm_$r.json)"
done
for r in va vb va2 vb2; do
  if [[ $r == va* ]]; then export DMP_XL_BM=0; else export DMP_XL_BM=-1; fi
  timeout -k 10 200 python bench.py --model vit_b_16 --batch-size 256 --steps 10 --warmup 5 > gpurun_out/bm_$r.json 2>gpurun_out/bm_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/bm_$r.json)"
done
