set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
js() { python -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms_per_step"], d["value"])' $1; }
timeout -k 10 200 python bench.py > gpurun_out/fin_r50.json 2>gpurun_out/fin_r50.err || exit 1
echo "r50 bs2048 $(js gpurun_out/fin_r50.json)"
timeout -k 10 200 python bench.py --batch-size 256 --steps 30 --warmup 10 > gpurun_out/fin_r50_256.json 2>gpurun_out/fin_r50_256.err || exit 1
echo "r50 bs256 $(js gpurun_out/fin_r50_256.json)"
timeout -k 10 200 python bench.py --model vit_b_16 --steps 30 --warmup 10 > gpurun_out/fin_vit.json 2>gpurun_out/fin_vit.err || exit 1
echo "vit $(js gpurun_out/fin_vit.json)"
timeout -k 10 200 python bench.py --model mobilenetv2 --steps 40 --warmup 10 > gpurun_out/fin_mnv2.json 2>gpurun_out/fin_mnv2.err || exit 1
echo "mnv2 $(js gpurun_out/fin_mnv2.json)"
timeout -k 10 200 python bench.py > gpurun_out/fin_r50b.json 2>gpurun_out/fin_r50b.err || exit 1
echo "r50 bs2048 again $(js gpurun_out/fin_r50b.json)"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_tr2048 -- python bench.py --steps 6 --warmup 4 > gpurun_out/fin_tr2048.log 2>&1 || exit 1
echo traced
