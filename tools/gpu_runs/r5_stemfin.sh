set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_stem.py tests/test_gpu_parity_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_stemfin.log 2>&1 || { tail -40 gpurun_out/t_stemfin.log; exit 1; }
tail -2 gpurun_out/t_stemfin.log
for r in a b; do
  timeout -k 10 200 python bench.py > gpurun_out/sf_$r.json 2>gpurun_out/sf_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/sf_$r.json)"
  timeout -k 10 200 python bench.py --batch-size 256 --steps 30 --warmup 10 > gpurun_out/sf256_$r.json 2>gpurun_out/sf256_$r.err || exit 1
  echo "256$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/sf256_$r.json)"
done
