"""Does a captured hipGraph run independent branches concurrently on MI355X?

Captures N tiny kernels (a) on one stream, (b) split over two forked streams
joined at the end, and times replays of each.  If (b) replays in about half
of (a), graph branches overlap, and side-stream work inside a capture (the
pipeline's weight gradients, parallel/pipeline.py) hides behind the main
chain.  usage: python tools/graph_branch_probe.py [--n 400] [--numel 4096]
"""
import argparse

import torch


def capture(n, numel, branches):
    xs = [torch.zeros(numel, device="cuda") for _ in range(branches)]
    streams = [torch.cuda.Stream() for _ in range(branches)]
    cap = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    cap.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=cap):
        for s in streams[1:]:
            s.wait_stream(cap)
        for i in range(n // branches):
            for b in range(branches):
                if b == 0:
                    xs[0].add_(1.0)
                else:
                    with torch.cuda.stream(streams[b]):
                        xs[b].add_(1.0)
        for s in streams[1:]:
            cap.wait_stream(s)
    return g, xs


def timed(g, reps=20):
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--numel", type=int, default=4096)
    a = ap.parse_args()
    for branches in (1, 2, 4):
        g, xs = capture(a.n, a.numel, branches)
        ms = timed(g)
        ok = all(float(x[0]) == (a.n // branches) * 21 for x in xs)
        print(f"branches {branches}: {a.n} kernels {ms:.3f} ms per replay, {1000 * ms / a.n:.2f} us per kernel"
              f"{'' if ok else ' WRONG RESULT'}", flush=True)


if __name__ == "__main__":
    main()
