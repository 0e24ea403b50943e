#!/usr/bin/env python3
"""Headline benchmark: ResNet-50 DDP bf16 training throughput (images/sec, whole node).

BASELINE.json metric: "images/sec (whole node) ResNet-50 DDP bf16 at 1/2/4/8
MI355X".  One process per GPU (torchrun for N>1), synthetic 3x224x224 inputs
and random-init weights (no datasets / checkpoints are available offline),
fixed per-GPU batch (weak scaling; ResNet-50 default 2048 images per GPU --
measured on 1x MI355X: 7607 img/s at 128, 8339 at 192, 8866 at 256, 9279 at
384, 9600-9744 at 512, 9948 at 768 (round 1); round 2: 11491-11818 at 1024
(40 GB peak), 11956-12155 at 2048 (80 GB peak, profiles/raw_r2/bench_bs*.log);
the 288 GB of HBM hold it easily, the activations of 3.3 GB per tensor are
checked for offset wrap by tests/test_gpu_bigbatch.py, and a bigger per-GPU share
also amortises the fixed gradient all-reduce).  Every timed step is a full training step:
forward, fp32 cross-entropy, backward with the native C++ reducer doing
bucketed RCCL all-reduces (25 MB buckets, ncclAvg) overlapped with backward,
one fused flat-SGD (momentum 0.9, wd 1e-4) launch per dtype group.

  python bench.py --gpus N --steps K --warmup W          (spawns N rank processes itself)
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Other BASELINE.json configs:
  DP (scatter/replicate/gather, one process): python bench.py --parallel dp --gpus N
  DDP + SyncBatchNorm:                        ... bench.py --parallel syncbn --gpus N
  ViT-B/16 DDP:                               ... bench.py --model vit_b_16   (256 per GPU)
  MobileNetV2 CIFAR pipeline (reference MP):  python bench.py --parallel pipe --model mobilenetv2
                                              --gpus 4 --batch-size 512 [--schedule naive|gpipe|1f1b]
  ResNet-18 CPU/gloo plumbing (ws 2):         torchrun --nproc-per-node 2 bench.py --device cpu
                                              --model resnet18 --dtype fp32 --batch-size 8
                                              --steps 2 --warmup 1 --no-channels-last

Rank 0 prints ONE JSON line.  Time = max over ranks of the K-step wall time,
bracketed by a barrier + device synchronize on both sides.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_model_parallel_amd.comm.rccl import default_communicator  # noqa: E402
from distributed_model_parallel_amd.models import INPUT_SHAPES  # noqa: E402
from distributed_model_parallel_amd.train.cli import start_watchdog  # noqa: E402
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state  # noqa: E402
from distributed_model_parallel_amd.utils.profiling import (  # noqa: E402
    enable_phase_timing, phase_summary, trace_range)
from distributed_model_parallel_amd.utils import gemm_tuning, miopen_db  # noqa: E402
from distributed_model_parallel_amd.utils.env import (  # noqa: E402
    count_gpus_without_hip, destroy_distributed, init_distributed)
from distributed_model_parallel_amd.utils.precision import parse_dtype  # noqa: E402

# per-GPU batch defaults (measured throughput curves: module docstring, README)
DEFAULT_BATCH = {"resnet50": 2048, "vit_b_16": 256, "mobilenetv2": 512}
BASELINE_VALUE = None  # BASELINE.json "published": {} -- no reference images/sec figure exists
# The reference's only throughput numbers (Readme.md:283-292): MobileNetV2 CIFAR
# time/batch -> images/sec, keyed (parallel, n_gpus, global batch).
REFERENCE_MNV2 = {("pipe", 4, 512): 512 / 1.616, ("dp", 4, 512): 512 / 0.396,
                  ("pipe", 2, 256): 256 / 0.772, ("dp", 2, 256): 256 / 0.363}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Launch n rank processes of this script (one per GPU) like the reference's
    ``mp.spawn(main_worker, nprocs=world_size)`` (model_parallel.py:160-162).

    Runs BEFORE anything touches the GPU in this parent (it only counts
    devices), children get the torchrun environment on 127.0.0.1; a failing
    rank takes the others down.  Returns the worst exit code."""
    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
                WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), DMP_BENCH_SPAWNED="1")
    procs = []
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # one rank died: the rest would hang in a collective
                    q.terminate()
        time.sleep(0.2)
    return rc


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--batch-size", type=int, default=None,
                    help="per-GPU batch (default: %s)" % DEFAULT_BATCH)
    ap.add_argument("--image-size", type=int, default=None, help="default: the model's native size")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--parallel", default="ddp", choices=["ddp", "syncbn", "dp", "pipe", "none"])
    ap.add_argument("--micro-batches", type=int, default=8, help="--parallel pipe")
    ap.add_argument("--schedule", default="1f1b", choices=["naive", "gpipe", "1f1b"],
                    help="--parallel pipe (naive = the reference's one-batch serial ring)")
    ap.add_argument("--partition", default="balanced", choices=["balanced", "reference"],
                    help="--parallel pipe stage cut")
    ap.add_argument("--bucket-cap-mb", type=float, default=25.0)
    ap.add_argument("--first-bucket-mb", type=float, default=1.0)
    ap.add_argument("--no-channels-last", action="store_true")
    ap.add_argument("--miopen-benchmark", type=int, default=1,
                    help="MIOpen find mode for the convs left on MIOpen (first step pays the search)")
    ap.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"],
                    help="cpu: gloo plumbing run (BASELINE config 1), fp32 recommended")
    ap.add_argument("--graph", action="store_true",
                    help="replay the whole training step as one captured hipGraph")
    ap.add_argument("--lr", type=float, default=None,
                    help="SGD learning rate (default 0.1 for CNNs, 0.005 for ViT: plain SGD at 0.1 "
                         "diverges on a transformer, which would make the reported loss meaningless)")
    ap.add_argument("--miopen-db", default="use",
                    choices=["use", "refresh", "off"],
                    help="seed MIOpen's find/perf db from profiles/miopen/ (use), also write new "
                         "entries back (refresh), or start empty (off); see utils/miopen_db.py")
    ap.add_argument("--dp-replicas", type=int, default=1,
                    help="--parallel dp: replicas per GPU; K>1 aliases K replicas onto each device so "
                         "scatter / replicate / parallel_apply / gather / reduce-add all execute even "
                         "on one GPU (the per-GPU batch is split K ways)")
    ap.add_argument("--dp-graphs", action="store_true",
                    help="--parallel dp: run every replica's forward / backward as captured hipGraphs "
                         "(parallel/dp_graphs.py) instead of Python threads")
    ap.add_argument("--no-pipe-graphs", action="store_true",
                    help="--parallel pipe: run the micro-batches eagerly instead of on captured stage graphs")
    ap.add_argument("--phase-times", action="store_true",
                    help="record HIP events around the DataParallel phases and report their GPU "
                         "ms per step in the JSON (config.phase_ms_per_step)")
    ap.add_argument("--single-rank-comm", action="store_true",
                    help="run the DDP bucket all-reduces and SyncBN moment all-reduces through RCCL "
                         "even at world size 1 (measures their cost on one GPU)")
    ap.add_argument("--checkpoint-segments", type=int, default=0, metavar="K",
                    help="activation checkpointing: recompute the block trunk in K segments in "
                         "backward (the reference's '2048(checkpoint)' runs, Readme.md:168,192)")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--watchdog", type=float, default=None, metavar="SECONDS",
                    help="exit 1 when the collective stream is stuck this long (default 900 s for "
                         "multi-rank GPU runs without --graph, 0 = off)")
    ap.add_argument("--trace-steps", action="store_true", help="diagnostic: time each warmup step")
    ap.add_argument("--gemm-tuning", default="use",
                    choices=["use", "tune", "off"],
                    help="library-GEMM solutions from profiles/tunableop/<model>_gfx950.csv "
                         "(use), re-tune and write that file (tune), or library defaults (off)")
    args = ap.parse_args()
    if args.batch_size is None:
        args.batch_size = DEFAULT_BATCH.get(args.model, 256)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.parallel != "dp":
        # no launcher: become one (before any GPU call in this process)
        # counted from the environment / KFD topology: this launcher never touches HIP
        seen = count_gpus_without_hip() if args.device != "cpu" else None
        if seen is not None and seen < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but only {seen} GPUs visible")
        if args.device == "cpu":  # gloo plumbing run: do not oversubscribe the host
            os.environ.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // args.gpus)))
        return spawn_ranks(args.gpus, sys.argv[1:])

    if args.single_rank_comm:
        os.environ["DMP_SINGLE_RANK_COMM"] = "1"
    use_gpu = None if args.device == "auto" else args.device == "cuda"
    env = init_distributed(use_gpu=use_gpu)
    if args.parallel != "dp" and env.world_size != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={env.world_size}: the launcher and the "
                         "flag disagree")
    torch.backends.cudnn.benchmark = bool(args.miopen_benchmark)
    if env.device.type == "cuda":
        miopen_db.seed(args.miopen_db)  # before the first conv creates the MIOpen handle
    dev = env.device
    tuning_file = gemm_tuning.configure(args.gemm_tuning, args.model) if dev.type == "cuda" else None
    cfg = StepConfig(model=args.model, batch_size=args.batch_size, image_size=args.image_size,
                     dtype=parse_dtype(args.dtype), channels_last=not args.no_channels_last,
                     parallel=args.parallel, bucket_cap_mb=args.bucket_cap_mb,
                     first_bucket_mb=args.first_bucket_mb,
                     dp_devices=args.gpus if args.parallel == "dp" else 1,
                     dp_replicas=args.dp_replicas, graph=args.graph,
                     lr=args.lr if args.lr is not None else (0.005 if args.model.startswith("vit") else 0.1),
                     micro_batches=args.micro_batches, schedule=args.schedule, partition=args.partition,
                     checkpoint_segments=args.checkpoint_segments, dp_graphs=args.dp_graphs,
                     pipe_graphs=not args.no_pipe_graphs)
    if args.parallel == "dp" and env.world_size > 1:
        raise SystemExit("--parallel dp is single-process multi-GPU: run `python bench.py --parallel dp "
                         "--gpus N` without torchrun")
    st = build_train_state(cfg, dev)
    comm = default_communicator(dev)
    wd = args.watchdog if args.watchdog is not None else (
        900.0 if env.world_size > 1 and dev.type == "cuda" and not args.graph else 0.0)
    dog = start_watchdog(wd, env)

    (_, img_h, _), _ = INPUT_SHAPES[args.model]
    image_size = args.image_size or img_h

    t_warm0 = time.time()
    first_step_ms = None
    for i in range(args.warmup):
        ts = time.perf_counter()
        loss = st.step()
        if i == 0 or (args.trace_steps and env.is_main):
            torch.cuda.synchronize() if dev.type == "cuda" else None
            ms = 1e3 * (time.perf_counter() - ts)
            if i == 0:
                first_step_ms = ms
            if env.is_main:
                print(f"[bench] warmup step {i} {ms:.1f} ms (t={time.time() - t_warm0:.1f}s) "
                      f"loss={loss.item():.4f}", file=sys.stderr, flush=True)
    comm.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if args.phase_times:
        enable_phase_timing()
        if args.parallel == "dp":
            from distributed_model_parallel_amd.parallel.data_parallel import reset_host_times
            reset_host_times()
    # per-bucket all-reduce timing of every timed backward (DDP only; a captured
    # graph replays without the reducer's host-side launches, so not there)
    timed_comm = hasattr(st.wrapped, "enable_comm_timing") and not args.graph
    if timed_comm:
        st.wrapped.enable_comm_timing(True)
    from distributed_model_parallel_amd.utils import routes
    routes0 = routes.route_counts()
    bcast0 = getattr(st.wrapped, "buffer_broadcasts", None)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        with trace_range("bench.step"):
            loss = st.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    elapsed = time.perf_counter() - t0
    rank_ms = 1000.0 * elapsed / args.steps
    elapsed = comm.max_scalar(elapsed)
    # where DDP time goes (the reference's question, Readme.md:10-15 / 145-157):
    # the last timed backward's per-bucket all-reduce ms and exposed comm tail,
    # and the spread of the per-rank step times (a slow rank shows here)
    ddp_comm = None
    if timed_comm:
        ddp_comm = st.wrapped.comm_timing()
        st.wrapped.enable_comm_timing(False)
        if "exposed_tail_ms" in ddp_comm:
            ddp_comm["exposed_tail_ms_max_over_ranks"] = round(comm.max_scalar(ddp_comm["exposed_tail_ms"]), 3)
    rank_step = {"max": round(comm.max_scalar(rank_ms), 3), "min": round(-comm.max_scalar(-rank_ms), 3)}
    final_loss = float(loss.item())
    step_routes = {k: round(v / args.steps, 2) for k, v in
                   sorted(routes.diff(routes.route_counts(), routes0).items())}
    phases = {k: {"ms_per_step": round(v["ms"] / args.steps, 3), "calls_per_step": v["calls"] / args.steps}
              for k, v in phase_summary().items()} if args.phase_times else None
    dp_host = None
    if args.parallel == "dp" and args.phase_times:
        from distributed_model_parallel_amd.parallel import data_parallel as _dpm
        ht = _dpm.HOST_TIMES
        if ht["applies"]:
            dp_host = {"apply_ms_per_step": round(ht["apply_ms"] / args.steps, 3),
                       "replicas": {str(i): {k: round(v / args.steps, 3) for k, v in r.items()}
                                    for i, r in sorted(ht["replicas"].items())}}

    # multi-rank facts the gloo rehearsal (tests/test_bench_multirank_cpu.py) checks:
    # every rank holds the same (rebuilt) bucket layout -- RCCL would deadlock on a
    # mismatch -- and module buffers cost one broadcast per dtype group per forward
    ddp_facts = None
    if hasattr(st.wrapped, "bucket_summary"):
        ddp_facts = st.wrapped.bucket_summary()
        dig = float(ddp_facts["digest"])
        ddp_facts["same_on_all_ranks"] = comm.max_scalar(dig) == -comm.max_scalar(-dig)
        ddp_facts["buffer_broadcasts_per_step"] = (st.wrapped.buffer_broadcasts - bcast0) / args.steps
        ddp_facts["buffer_dtype_groups"] = len(st.wrapped._buffers_flat or [])

    import torch.distributed as dist
    n = dist.get_world_size()
    if args.parallel == "dp" and dev.type == "cuda":
        n = args.gpus  # one process driving N GPUs
    # pipe: the batch is the whole pipeline's batch; data parallel: per GPU
    global_batch = args.batch_size if args.parallel == "pipe" else args.batch_size * n
    img_s = global_batch * args.steps / elapsed
    par = {"ddp": "ddp", "syncbn": "ddp-syncbn", "dp": "dp-single-process", "pipe": "pipe",
           "none": "none"}[args.parallel]
    metric = f"images/sec (whole node) {'ResNet-50' if args.model == 'resnet50' else args.model} " \
             f"{'DDP' if args.parallel in ('ddp', 'syncbn') else args.parallel.upper()} {args.dtype}"
    ref = REFERENCE_MNV2.get((args.parallel, n, global_batch)) if args.model == "mobilenetv2" else None
    ref = ref or BASELINE_VALUE
    result = {
        "metric": metric,
        "value": round(img_s, 2),
        "unit": "images/sec",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.parallel == "pipe" else "weak",
        "vs_baseline": round(img_s / ref, 3) if ref else None,
        "dtype": args.dtype,
        "data": "synthetic (random 3x%dx%d inputs, random labels, random-init weights)"
                % (image_size, image_size),
        "config": {
            "model": args.model,
            "device": dev.type,
            "global_batch": global_batch,
            "per_gpu_batch": args.batch_size,
            "seq_len": None,
            "image_size": image_size,
            "parallelism": f"{par}{n}",
            **({"dp_replicas_per_gpu": args.dp_replicas, "dp_graphs": args.dp_graphs,
                "dp_device_ids": getattr(st.wrapped, "device_ids", None)} if args.parallel == "dp" else {}),
            **({"phase_ms_per_step": phases} if phases is not None else {}),
            **({"dp_host_ms_per_step": dp_host} if dp_host is not None else {}),
            "single_rank_comm": bool(args.single_rank_comm),
            "ranks": dist.get_world_size(),
            "rccl_ranks": comm.size if comm.native is not None else None,
            "launcher": "bench-spawn" if os.environ.get("DMP_BENCH_SPAWNED") else
            ("torchrun" if "TORCHELASTIC_RUN_ID" in os.environ else "single"),
            "optimizer": type(st.optimizer).__name__ + ("(fp32 master)" if args.dtype != "fp32" else ""),
            "sync_bn": args.parallel == "syncbn",
            "bucket_cap_mb": args.bucket_cap_mb,
            "channels_last": not args.no_channels_last,
            "grad_comm": getattr(st.wrapped, "comm_backend", None),
            **({"micro_batches": args.micro_batches, "schedule": args.schedule,
                "stage_partition": st.wrapped.partition,
                "stage_graphs": bool(st.wrapped._graphs)} if args.parallel == "pipe" else {}),
            **({"reference_images_per_sec": round(ref, 1)} if ref else {}),
            "hip_graph": args.graph,
            "checkpoint_segments": args.checkpoint_segments,
            "watchdog_s": wd,
            "gemm_tuning": os.path.relpath(tuning_file, os.path.dirname(os.path.abspath(__file__)))
            if tuning_file else args.gemm_tuning if args.gemm_tuning != "use" else None,
            # the untimed first step pays MIOpen's solver search for the convs still on
            # MIOpen unless its find db is seeded from profiles/miopen/ (utils/miopen_db.py)
            "miopen_db": args.miopen_db if dev.type == "cuda" else None,
            "first_step_ms": round(first_step_ms, 1) if first_step_ms is not None else None,
            "final_loss": round(final_loss, 4),
            "routes_per_step": step_routes,
            **({"ddp_buckets": ddp_facts} if ddp_facts is not None else {}),
            **({"ddp_comm": ddp_comm} if ddp_comm is not None else {}),
            "rank_step_ms": rank_step,
            "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 1)
            if dev.type == "cuda" else None,
        },
    }
    if env.is_main:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dog is not None:
        dog.stop()
    destroy_distributed()
    return 0


if __name__ == "__main__":
    sys.exit(main())
