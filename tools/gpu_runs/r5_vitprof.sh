set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_trvit -- python bench.py --model vit_b_16 --steps 6 --warmup 4 > gpurun_out/fin_trvit.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_trmnv2 -- python bench.py --model mobilenetv2 --steps 8 --warmup 4 > gpurun_out/fin_trmnv2.log 2>&1 || exit 1
echo traced
