set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr2048 -- python bench.py --steps 6 --warmup 4 > gpurun_out/tr2048.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr256 -- python bench.py --batch-size 256 --steps 12 --warmup 8 > gpurun_out/tr256.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trvit -- python bench.py --model vit_b_16 --batch-size 256 --steps 8 --warmup 5 > gpurun_out/trvit.log 2>&1 || exit 1
timeout -k 10 400 python tools/step_roofline.py --batch-size 2048 > gpurun_out/roof2048.md 2> gpurun_out/roof2048.err || exit 1
