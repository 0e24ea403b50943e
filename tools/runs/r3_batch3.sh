#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r3h; mkdir -p $O
export PYTHONUNBUFFERED=1
run() { local name=$1; shift; echo "== $name"; timeout -k 10 ${T:-300} "$@" > $O/$name.log 2>&1; local rc=$?; tail -2 $O/$name.log; return $rc; }
T=500 DMP_CONVERGENCE_OUT=$O/convergence.json run conv python -u -m pytest tests/test_gpu_convergence.py -x -q --timeout 400 --timeout-method thread
T=200 run halobench python tools/halo_bench.py --batch 2048 &&
T=300 run dp4_256 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 30 --warmup 10 --phase-times &&
T=300 run mnv2 python bench.py --model mobilenetv2 --steps 50 --warmup 10 &&
T=300 run mnv2_graph python bench.py --model mobilenetv2 --steps 50 --warmup 10 --graph &&
T=300 run r50_256 python bench.py --batch-size 256 --steps 30 --warmup 10 &&
T=300 run r50_256_graph python bench.py --batch-size 256 --steps 30 --warmup 10 --graph &&
T=300 run prof_mnv2 rocprofv3 --kernel-trace --stats -d $O/prof_mnv2 -o p --output-format csv -- python3 bench.py --model mobilenetv2 --steps 6 --warmup 3 &&
T=300 run prof_mnv2_graph rocprofv3 --kernel-trace --stats -d $O/prof_mnv2g -o p --output-format csv -- python3 bench.py --model mobilenetv2 --steps 6 --warmup 3 --graph
