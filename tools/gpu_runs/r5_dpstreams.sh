set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_data_parallel.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_dps.log 2>&1 || { tail -40 gpurun_out/t_dps.log; exit 1; }
tail -2 gpurun_out/t_dps.log
for r in s1 s0 s1b s0b; do
  case $r in s1*) export DMP_DP_ALIAS_STREAMS=1;; s0*) export DMP_DP_ALIAS_STREAMS=0;; esac
  timeout -k 10 200 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --phase-times > gpurun_out/dps_$r.json 2>gpurun_out/dps_$r.err || exit 1
  echo "$r $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/dps_$r.json)"
done
