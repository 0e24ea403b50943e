set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 3 --phase-times > gpurun_out/dp_eager.log 2>&1 &&
timeout -k 10 300 python -u bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 3 --dp-graphs > gpurun_out/dp_graphs.log 2>&1 &&
timeout -k 10 300 python -u bench.py --batch-size 256 --steps 10 --warmup 3 > gpurun_out/ddp256.log 2>&1 &&
timeout -k 10 300 python -u bench.py --model mobilenetv2 --steps 10 --warmup 3 > gpurun_out/mnv2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mnv2_r6 -o run -- python -u bench.py --model mobilenetv2 --steps 4 --warmup 3 > gpurun_out/mnv2_prof.log 2>&1
