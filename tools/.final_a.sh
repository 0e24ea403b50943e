set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/pipe_bench.py --lib --epi --rounds 3 > gpurun_out/pipe_bench_r6.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model mobilenetv2 --graph --steps 10 --warmup 3 > gpurun_out/mnv2_graph.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch-size 256 --graph --steps 10 --warmup 3 > gpurun_out/r50_256_graph.log 2>&1 &&
timeout -k 10 300 python -u bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 3 > gpurun_out/dp_eager3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --parallel pipe --model mobilenetv2 --no-pipe-graphs --steps 5 --warmup 2 > gpurun_out/pipe_eager2.log 2>&1
