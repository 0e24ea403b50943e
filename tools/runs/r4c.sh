set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_data_parallel.py tests/test_gpu_checkpointing.py tests/test_gpu_bn_fold.py -m gpu > $O/r4c_tests.log 2>&1
rc=$?; tail -3 $O/r4c_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --phase-times > $O/r4c_dp4_eager.log 2>&1
rc=$?; tail -1 $O/r4c_dp4_eager.log | cut -c1-300; [ $rc -ge 124 ] && exit $rc
timeout -k 10 200 python bench.py --parallel dp --dp-replicas 4 --batch-size 256 --steps 10 --warmup 5 --dp-graphs > $O/r4c_dp4_graphs.log 2>&1
rc=$?; tail -1 $O/r4c_dp4_graphs.log | cut -c1-300; [ $rc -ge 124 ] && exit $rc
timeout -k 10 400 env DMP_CONVERGENCE_OUT=$O/r4c_conv.json python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_gpu_convergence.py -k "224" > $O/r4c_conv.log 2>&1
rc=$?; tail -3 $O/r4c_conv.log; exit 0
