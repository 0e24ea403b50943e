set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/xl_phase_trace.py > gpurun_out/xl_phase.md 2>&1 || { cat gpurun_out/xl_phase.md; exit 1; }
cat gpurun_out/xl_phase.md
T=tests/test_gpu_convergence.py::test_resnet50_224_training_covers_bench_routes_and_tracks_stock
DMP_CONVERGENCE_OUT=gpurun_out/conv_fold.json timeout -k 10 400 python -u -m pytest $T -x -q --timeout 380 --timeout-method thread > gpurun_out/conv_fold.log 2>&1; echo "fold rc=$?"
DMP_DISABLE=fuse_stem_wgrad DMP_CONVERGENCE_OUT=gpurun_out/conv_nofold.json timeout -k 10 400 python -u -m pytest $T -x -q --timeout 380 --timeout-method thread > gpurun_out/conv_nofold.log 2>&1; echo "nofold rc=$?"
