"""8-rank rehearsal of the multi-GPU paths on the CPU (gloo), through the same
``bench.py`` the driver launches at N = 8: ResNet-50 DDP,
ResNet-50 DDP + SyncBatchNorm and an 8-stage MobileNetV2 pipeline, tiny
images, fp32.  The 8-GPU runs themselves are the driver's; what is checked
here is the rank-count-dependent logic: every rank ends with the SAME rebuilt
bucket layout (RCCL would deadlock on a mismatch), module buffers cost one
broadcast per dtype group per forward, the SyncBN reducers and the 8-way
pipeline partition run end to end."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args) -> dict:
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "8",
                        "--dtype", "fp32", "--steps", "2", "--warmup", "2", *args],
                       capture_output=True, text=True, timeout=900, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def _check_ddp(d: dict) -> None:
    c = d["config"]
    assert d["n_gpus"] == 8 and c["ranks"] == 8 and c["launcher"] == "bench-spawn"
    assert c["grad_comm"] == "process_group"
    b = c["ddp_buckets"]
    assert b["same_on_all_ranks"] and b["rebuilt"], b
    # ResNet-50 fp32 gradients (102 MB) in 25 MB buckets after a 1 MB first cap
    assert 4 <= b["buckets"] <= 6 and abs(sum(b["bucket_mb"]) - 97.49) < 0.5, b
    assert b["buffer_broadcasts_per_step"] == b["buffer_dtype_groups"] == 2, b
    assert c["final_loss"] == c["final_loss"]  # not NaN
    # communication accounting: per-bucket all-reduce
    # times of the last timed backward, the exposed tail and the rank spread
    cc = c["ddp_comm"]
    assert cc["backend"] == "process_group" and cc["source"] == "host_clock", cc
    n = b["buckets"]
    assert cc["buckets_timed"] == n and len(cc["ready_to_done_ms"]) == n and len(cc["allreduce_ms"]) == n, cc
    assert all(x >= 0 for x in cc["ready_to_done_ms"] + cc["allreduce_ms"]) and cc["exposed_tail_ms"] >= 0, cc
    assert all(a <= r + 1e-6 for a, r in zip(cc["allreduce_ms"], cc["ready_to_done_ms"])), cc
    assert cc["exposed_tail_ms_max_over_ranks"] >= cc["exposed_tail_ms"] - 1e-6, cc
    rs = c["rank_step_ms"]
    assert 0 < rs["min"] <= rs["max"] <= d["ms_per_step"] + 1e-3, rs


def test_resnet50_ddp_8_ranks():
    _check_ddp(_bench("--model", "resnet50", "--image-size", "32", "--batch-size", "2"))


def test_resnet50_ddp_syncbn_8_ranks():
    d = _bench("--model", "resnet50", "--parallel", "syncbn", "--image-size", "32", "--batch-size", "2")
    _check_ddp(d)
    assert d["config"]["sync_bn"]


def test_mobilenetv2_pipeline_8_stages():
    d = _bench("--model", "mobilenetv2", "--parallel", "pipe", "--batch-size", "16", "--micro-batches", "8")
    c = d["config"]
    parts = c["stage_partition"]
    assert len(parts) == 8 and parts[0][0] == 0 and parts[-1][1] == 20
    assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))
    assert c["schedule"] == "1f1b" and c["ranks"] == 8
    assert c["final_loss"] == c["final_loss"]
