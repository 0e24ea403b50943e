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
