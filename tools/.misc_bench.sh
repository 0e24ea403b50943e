set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 3 > gpurun_out/dp_eager2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model vit_b_16 --steps 10 --warmup 3 > gpurun_out/vit.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model mobilenetv2 --graph --steps 10 --warmup 3 > gpurun_out/mnv2_graph.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch-size 256 --graph --steps 10 --warmup 3 > gpurun_out/r50_256_graph.log 2>&1 &&
timeout -k 10 300 python -u bench.py --parallel pipe --model mobilenetv2 --no-pipe-graphs --steps 5 --warmup 2 > gpurun_out/pipe_eager.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vit_r6 -o run -- python -u bench.py --model vit_b_16 --steps 4 --warmup 3 > gpurun_out/vit_prof.log 2>&1
