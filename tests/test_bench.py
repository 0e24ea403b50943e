"""bench.py contract on CPU/gloo: `--gpus N` without a launcher spawns N rank
processes itself (reference: mp.spawn, model_parallel.py:160-162) and rank 0
prints ONE JSON line whose n_gpus is the real world size; `--parallel pipe`
runs the pipeline across those ranks."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--dtype", "fp32",
                        "--no-channels-last", "--steps", "1", "--warmup", "1", *extra],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    err = "\n".join(l for l in r.stderr.splitlines() if "hostname of the client" not in l and "[Gloo]" not in l)
    assert r.returncode == 0, err[-6000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_spawns_ranks_ddp():
    res = _run("--gpus", "2", "--model", "resnet18", "--batch-size", "2", "--image-size", "32")
    assert res["n_gpus"] == 2 and res["config"]["ranks"] == 2
    assert res["config"]["launcher"] == "bench-spawn"
    assert res["config"]["global_batch"] == 4 and res["scaling"] == "weak"
    assert res["config"]["grad_comm"] == "process_group"


def test_bench_pipe_two_stages():
    res = _run("--gpus", "2", "--parallel", "pipe", "--model", "mobilenetv2", "--batch-size", "8",
               "--micro-batches", "2", "--schedule", "gpipe")
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "pipe2"
    assert res["config"]["global_batch"] == 8 and res["scaling"] == "strong"
    assert len(res["config"]["stage_partition"]) == 2
    assert res["ms_per_step"] > 0


def test_bench_syncbn_four_ranks():
    """DDP + SyncBatchNorm through bench.py on 4 gloo ranks: the moment
    all-reduces run across ranks (rehearse more ranks on CPU)."""
    res = _run("--gpus", "4", "--parallel", "syncbn", "--model", "resnet18", "--batch-size", "2",
               "--image-size", "32")
    assert res["n_gpus"] == 4 and res["config"]["ranks"] == 4
    assert res["config"]["sync_bn"] is True and res["config"]["parallelism"] == "ddp-syncbn4"
    assert res["config"]["global_batch"] == 8


def test_bench_pipe_reference_four_way_naive():
    """The reference's own experiment: MobileNetV2 cut 4 ways exactly as
    model_parallel.py:103,129,144 does, naive (one batch, serial ring) schedule."""
    res = _run("--gpus", "4", "--parallel", "pipe", "--model", "mobilenetv2", "--batch-size", "8",
               "--micro-batches", "1", "--schedule", "naive", "--partition", "reference")
    assert res["n_gpus"] == 4 and res["config"]["parallelism"] == "pipe4"
    assert res["config"]["schedule"] == "naive" and len(res["config"]["stage_partition"]) == 4
    assert res["ms_per_step"] > 0


def test_bench_ddp_label_and_single_rank_comm_flag():
    res = _run("--model", "resnet18", "--batch-size", "2", "--image-size", "32", "--single-rank-comm")
    assert res["config"]["parallelism"] == "ddp1" and res["config"]["single_rank_comm"] is True
    # at world size 1 the forced path goes through the process-group backend on CPU
    assert res["config"]["grad_comm"] == "process_group"
