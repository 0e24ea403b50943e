set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/torch_op_sources.py --model mobilenetv2 --batch-size 512 --steps 3 > gpurun_out/mnv2_src3.md 2>gpurun_out/mnv2_src3.err || { tail -20 gpurun_out/mnv2_src3.err; exit 1; }
grep "^|" gpurun_out/mnv2_src3.md | head -8
