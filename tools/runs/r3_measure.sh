#!/bin/bash
# Round-3 measurement pass on one MI355X: GPU suite, then the bench lines the
# README claims (each step time-limited; stop at the first failure).
set -u
O=gpurun_out/r3a
mkdir -p $O
export PYTHONUNBUFFERED=1
run() { local name=$1; shift; echo "== $name: $*"; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log; return $rc; }
T=600 run gputests python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
T=300 run bench_ddp python bench.py --steps 20 --warmup 5 &&
T=300 run bench_ddp_rccl python bench.py --steps 20 --warmup 5 --single-rank-comm &&
T=300 run bench_syncbn_rccl python bench.py --parallel syncbn --steps 20 --warmup 5 --single-rank-comm &&
T=300 run bench_dp4 python bench.py --parallel dp --dp-replicas 4 --steps 20 --warmup 5 --phase-times &&
T=300 run bench_ddp256 python bench.py --batch-size 256 --steps 30 --warmup 10 &&
T=300 run bench_ddp256_rccl python bench.py --batch-size 256 --steps 30 --warmup 10 --single-rank-comm &&
T=300 run bench_dp4_256 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 30 --warmup 10 --phase-times
