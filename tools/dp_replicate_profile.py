"""Host-time breakdown of DataParallel's replicate() for ResNet-50 (bf16,
channels-last) on K aliased replicas of one GPU: cProfile of the main-thread
call, the part of a DP step that runs before any replica starts.

usage: python tools/dp_replicate_profile.py [--replicas 4] [--iters 20]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from distributed_model_parallel_amd.models import resnet50
    from distributed_model_parallel_amd.parallel import data_parallel as dp
    from distributed_model_parallel_amd.utils.precision import cast_model
    net = cast_model(resnet50().cuda(), torch.bfloat16).to(memory_format=torch.channels_last)
    devs = [0] * a.replicas
    cache = {}
    for _ in range(3):
        dp.replicate(net, devs, cache=cache).release()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        dp.replicate(net, devs, cache=cache).release()
    torch.cuda.synchronize()
    print(f"replicate: {1e3 * (time.perf_counter() - t) / a.iters:.2f} ms per call (host + queued copies)")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.iters):
        dp.replicate(net, devs, cache=cache).release()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
