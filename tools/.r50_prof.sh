set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_r6 -o run -- python -u bench.py --steps 4 --warmup 3 > gpurun_out/r50_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_256_r6 -o run -- python -u bench.py --batch-size 256 --steps 6 --warmup 3 > gpurun_out/r50_256_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit_r6 -o run -- python -u bench.py --model vit_b16 --steps 4 --warmup 3 > gpurun_out/vit_prof.log 2>&1
