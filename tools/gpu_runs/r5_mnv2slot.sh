set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_mnv2_block.py tests/test_gpu_models.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_mslot.log 2>&1 || { tail -40 gpurun_out/t_mslot.log; exit 1; }
tail -2 gpurun_out/t_mslot.log
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
for r in new old new2 old2 new3 old3; do
  case $r in old*) export DMP_MNV2_NOSLOT=1;; *) unset DMP_MNV2_NOSLOT;; esac
  timeout -k 10 200 python bench.py --model mobilenetv2 --steps 40 --warmup 10 > gpurun_out/ms_$r.json 2>gpurun_out/ms_$r.err || exit 1
  echo "$r mnv2 $(js gpurun_out/ms_$r.json)"
done
