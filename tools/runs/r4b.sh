set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attention.py > $O/r4b_attn_tests.log 2>&1 && \
timeout -k 10 120 env B=256 python -u tools/attn_bench.py > $O/r4b_attn.log 2>&1 && \
timeout -k 10 300 python -u tools/step_roofline.py > $O/r4b_roofline_r50.md 2> $O/r4b_roofline_r50.err && \
timeout -k 10 300 python -u tools/step_roofline.py --model vit_b_16 > $O/r4b_roofline_vit.md 2> $O/r4b_roofline_vit.err && \
timeout -k 10 300 python -u tools/step_roofline.py --batch-size 256 > $O/r4b_roofline_r50_256.md 2> $O/r4b_roofline_r50_256.err && \
timeout -k 10 300 python bench.py --batch-size 256 --steps 30 --warmup 10 > $O/r4b_b256.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r4b_prof256 -o prof --output-format csv -- python3 bench.py --batch-size 256 --steps 6 --warmup 3 > $O/r4b_prof256.log 2>&1
