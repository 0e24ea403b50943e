set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python bench.py --steps 10 --warmup 5 > gpurun_out/dps_head.json 2>/dev/null || exit 1
echo "head $(python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' gpurun_out/dps_head.json)"
for r in s0 s1 s0b s1b; do
  case $r in s1*) export DMP_DP_ALIAS_STREAMS=1;; s0*) export DMP_DP_ALIAS_STREAMS=0;; esac
  timeout -k 10 200 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 5 --warmup 3 --phase-times > gpurun_out/dps2_$r.json 2>gpurun_out/dps2_$r.err || exit 1
  python -c "
import json,sys; d=json.loads(open('gpurun_out/dps2_$r.json').read().strip().splitlines()[-1]); c=d['config']
print('$r', d['ms_per_step'], {k:round(v['ms_per_step'],1) for k,v in c.get('phase_ms_per_step',{}).items()})"
done
