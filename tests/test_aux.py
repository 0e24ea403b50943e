"""Auxiliary subsystems: activation checkpointing (D12), roctx ranges,
rank0_first, CLI smoke on CPU (pipeline via mp.spawn, DDP single process)."""
import os
import subprocess
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_model_parallel_amd.models import MobileNetV2
from distributed_model_parallel_amd.utils.checkpointing import CheckpointedSequential, checkpoint_sequential
from distributed_model_parallel_amd.utils.profiling import mark, trace_range

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_checkpoint_sequential_matches_plain_with_bn():
    torch.manual_seed(0)
    a = MobileNetV2().as_sequential()
    torch.manual_seed(0)
    b = MobileNetV2().as_sequential()
    x = torch.randn(4, 3, 32, 32)
    y = torch.randint(0, 10, (4,))
    F.cross_entropy(a(x), y).backward()
    F.cross_entropy(checkpoint_sequential(b, 4, x.clone()), y).backward()
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(p.grad, q.grad, atol=1e-5, rtol=1e-4, msg=n)
    for (n, s), t in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(s, t, msg=n)  # running stats updated exactly once


def test_checkpointed_sequential_module():
    m = CheckpointedSequential(nn.Linear(4, 4), nn.ReLU(), nn.Linear(4, 2), segments=2)
    x = torch.randn(3, 4, requires_grad=True)
    m(x).sum().backward()
    assert x.grad is not None


def test_trace_range_is_safe_without_gpu():
    with trace_range("test"):
        mark("inside")


def _cli(args, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONPATH=ROOT)
    env.pop("RANK", None)
    return subprocess.run([sys.executable, "-m", "distributed_model_parallel_amd.train.cli", *args],
                          cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_cli_pipeline_world2_cpu(tmp_path):
    r = _cli(["--parallel", "pipe", "--world-size", "2", "--arch", "mobilenetv2", "--synthetic",
              "-b", "16", "--epochs", "1", "--steps-per-epoch", "2", "--micro-batches", "2",
              "--schedule", "1f1b", "--log-dir", str(tmp_path / "log"),
              "--checkpoint", str(tmp_path / "ck" / "c.pth"), "-j", "0"])
    assert r.returncode == 0, r.stderr[-3000:]
    text = (tmp_path / "log" / "16.txt").read_text()
    assert "step:0" in text and "loss_train" in text
    assert (tmp_path / "ck" / "c.stage0.pth").exists() and (tmp_path / "ck" / "c.stage1.pth").exists()


def test_cli_ddp_single_process_cpu(tmp_path):
    env_port = str(29000 + os.getpid() % 1000)
    os.environ["MASTER_PORT"] = env_port
    r = _cli(["--parallel", "ddp", "--arch", "mobilenetv2", "--synthetic", "-b", "8", "--epochs", "2",
              "--steps-per-epoch", "2", "--log-dir", str(tmp_path / "log"), "-j", "0",
              "--checkpoint", str(tmp_path / "ck.pth")])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = (tmp_path / "log" / "ddp_8.txt").read_text().strip().splitlines()
    assert len(lines) == 2


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_cpu_plumbing_resnet18_ws2():
    """BASELINE.json config 1: ResNet-18 data-parallel plumbing on CPU / gloo, world size 2,
    synthetic 3x224x224, through the same bench.py the driver runs on MI355X."""
    import json
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--model", "resnet18",
           "--dtype", "fp32", "--batch-size", "2", "--steps", "1", "--warmup", "1", "--no-channels-last"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == 2 and res["config"]["global_batch"] == 4
    assert res["config"]["device"] == "cpu" and res["value"] > 0


def test_multinode_simulation_two_torchrun_nodes():
    """two `torchrun --nnodes 2 --node-rank {0,1}` launches on one host
    (rank != local_rank on node 1) running the DDP bench step over gloo."""
    import json
    port = str(_free_port())
    env = dict(os.environ, OMP_NUM_THREADS="2")
    procs = []
    for node in (0, 1):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "2", "--node-rank", str(node),
               "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port", port,
               os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "cpu", "--model", "resnet18",
               "--dtype", "fp32", "--batch-size", "2", "--image-size", "64", "--steps", "2", "--warmup", "1",
               "--no-channels-last"]
        procs.append(subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True))
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    line = [ln for ln in outs[0][0].splitlines() if ln.startswith("{")][-1]
    assert json.loads(line)["n_gpus"] == 2
    assert not [ln for ln in outs[1][0].splitlines() if ln.startswith("{")]  # only global rank 0 prints


def test_ddp_bucketing_at_world_64_with_fake_backend():
    """the `fake` process group exercises DDP construction and bucket
    assignment for ResNet-50 / ViT-B/16 at world size 64 without communication."""
    code = r'''
import torch, torch.distributed as dist
from torch.testing._internal.distributed.fake_pg import FakeStore
from distributed_model_parallel_amd.models import build_model
from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
dist.init_process_group("fake", store=FakeStore(), rank=5, world_size=64)
for name, cap in (("resnet50", 25.0), ("vit_b_16", 25.0)):
    m = build_model(name)
    ddp = DistributedDataParallel(m, bucket_cap_mb=cap, first_bucket_mb=1.0)
    sizes = [sum(ddp._params[i].numel() * ddp._params[i].element_size() for i in b)
             for b in ddp.reducer.buckets()]
    n = len(ddp._params)
    assert sorted(i for b in ddp.reducer.buckets() for i in b) == list(range(n))
    assert sizes[0] <= 1.0 * 2**20 + max(p.numel() * 4 for p in ddp._params)
    assert all(s <= cap * 2**20 + max(p.numel() * 4 for p in ddp._params) for s in sizes)
    print(name, len(sizes), [round(s / 2**20, 1) for s in sizes])
dist.destroy_process_group()
'''
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "resnet50" in r.stdout and "vit_b_16" in r.stdout


def test_miopen_db_seed(tmp_path, monkeypatch):
    """utils/miopen_db.py: the committed find db is copied to a private dir and
    MIOPEN_USER_DB_PATH points at it; a user-set path is left alone."""
    from distributed_model_parallel_amd.utils import miopen_db
    monkeypatch.delenv("MIOPEN_USER_DB_PATH", raising=False)
    monkeypatch.setenv("TMPDIR", str(tmp_path))
    d = miopen_db.seed("use")
    assert d is not None and os.environ["MIOPEN_USER_DB_PATH"] == d
    shipped = sorted(f.name for f in miopen_db.DB_DIR.glob("*.txt"))
    assert shipped and sorted(os.listdir(d)) == shipped
    assert any(n.endswith(".ufdb.txt") for n in shipped)
    monkeypatch.setenv("MIOPEN_USER_DB_PATH", "/somewhere/else")
    assert miopen_db.seed("use") is None
    assert os.environ["MIOPEN_USER_DB_PATH"] == "/somewhere/else"
    assert miopen_db.seed("off") is None
    for k in miopen_db.NAIVE_SOLVER_ENVS:
        assert os.environ[k] == "0"
        monkeypatch.delenv(k)


def test_miopen_db_entries_have_fast_solvers():
    """Every committed find-db problem has an implicit-GEMM solver besides the
    naive reference one, so dropping the naive solvers from find is safe for it."""
    from distributed_model_parallel_amd.utils import miopen_db
    n = 0
    for f in miopen_db.DB_DIR.glob("*.ufdb.txt"):
        for line in f.read_text().splitlines():
            key, sols = line.split("=", 1)
            names = [s.split(":")[0] for s in sols.split(";")]
            assert any("ImplicitGemm" in s for s in names), key
            n += 1
    assert n > 0


def _rank0_first_worker(rank, world):
    import time
    from distributed_model_parallel_amd.utils.debug import rank0_first
    with rank0_first():
        t_in = time.monotonic()
        if rank == 0:
            time.sleep(0.5)  # slow "preparation" on rank 0
        t_out = time.monotonic()
    return (t_in, t_out)


def test_rank0_first_orders_dataset_preparation():
    """SURVEY defect 6 (all ranks preparing ./data at once): the CLI builds its
    datasets under rank0_first -- every other rank enters only after rank 0 left."""
    from tests.dist_utils import run_world
    res = run_world(_rank0_first_worker, 3)
    r0_out = res[0][1]
    assert all(t_in >= r0_out - 1e-3 for t_in, _ in res[1:]), res
