set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
timeout -k 10 300 python bench.py --model mobilenetv2 --graph --steps 40 --warmup 10 > gpurun_out/mg.json 2>gpurun_out/mg.err || { tail -20 gpurun_out/mg.err; exit 1; }
echo "mnv2 graph $(js gpurun_out/mg.json)"
timeout -k 10 300 python bench.py --batch-size 256 --graph --steps 30 --warmup 10 > gpurun_out/rg.json 2>gpurun_out/rg.err || { tail -20 gpurun_out/rg.err; exit 1; }
echo "r50 bs256 graph $(js gpurun_out/rg.json)"
