set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stem.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_pool.log 2>&1 || { tail -40 gpurun_out/t_pool.log; exit 1; }
tail -2 gpurun_out/t_pool.log
echo new; timeout -k 10 120 python tools/pool_bn_bench.py
echo fwd1; DMP_POOL_FWD1=1 timeout -k 10 120 python tools/pool_bn_bench.py
echo old; DMP_NATIVE_SO=$PWD/ab_so/_C_old.so timeout -k 10 120 python tools/pool_bn_bench.py
echo new; timeout -k 10 120 python tools/pool_bn_bench.py
