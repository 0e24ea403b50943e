"""Cross-rank ordering of the two communicators of DDP + SyncBatchNorm
(VERDICT r3 weak 7 / next-round item 3d).

The ordering argument that rules out a cross-communicator deadlock
(distributed_model_parallel_amd/parallel/sync_batchnorm.py, "Ordering"):
every collective of both communicators is ENQUEUED by one host thread per
rank (forward: the module's own thread; backward: the autograd device thread,
which runs the SyncBN backward nodes AND the reducer's post-accumulate hooks
that launch the buckets, csrc/ddp/reducer.cpp launch_ready_prefix_locked), in
an order fixed by the (identical) autograd graph; so the interleaving of
SyncBN and bucket collectives in submission order is the same on every rank,
and a kernel of one communicator can only wait behind (on a shared hardware
queue) kernels that every peer also submitted before it.

This test records that interleaving on every rank of a gloo world and
requires it to be identical, over iterations that include the first-backward
bucket rebuild."""
import torch
import torch.nn.functional as F

from tests.dist_utils import run_world


def _worker(rank, world):
    import torch.distributed as dist
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.models import build_model
    from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
    from distributed_model_parallel_amd.parallel.sync_batchnorm import SyncBatchNorm
    log = []
    orig = Communicator.all_reduce

    def logged(self, t, op="sum", on_current_stream=False):
        log.append(("syncbn", int(t.numel())))
        return orig(self, t, op, on_current_stream)
    Communicator.all_reduce = logged
    try:
        torch.manual_seed(0)
        m = SyncBatchNorm.convert_sync_batchnorm(build_model("resnet18", num_classes=10))
        ddp = DistributedDataParallel(m, bucket_cap_mb=2.0, first_bucket_mb=0.5)

        def hook(state, bucket):
            log.append(("ddp", bucket.index()))
            fut = dist.all_reduce(bucket.buffer(), async_op=True).get_future()
            return fut.then(lambda f: f.value()[0].div_(world))
        ddp.register_comm_hook(None, hook)
        torch.manual_seed(100 + rank)
        seqs = []
        for _ in range(3):
            log.clear()
            x = torch.randn(2, 3, 32, 32)
            y = torch.randint(0, 10, (2,))
            F.cross_entropy(ddp(x), y).backward()
            seqs.append(list(log))
        return {"seqs": seqs, "buckets": len(ddp.reducer.buckets())}
    finally:
        Communicator.all_reduce = orig


def test_syncbn_and_bucket_collectives_interleave_identically_on_every_rank():
    res = run_world(_worker, 2)
    assert res[0]["buckets"] > 2
    for it, (a, b) in enumerate(zip(res[0]["seqs"], res[1]["seqs"])):
        assert any(k == "ddp" for k, _ in a) and any(k == "syncbn" for k, _ in a)
        assert a == b, f"iteration {it}: ranks submitted the two communicators' collectives in different orders"
        # buckets interleave with SyncBN backward all-reduces (overlap), not after them
        kinds = [k for k, _ in a]
        first_ddp = kinds.index("ddp")
        assert "syncbn" in kinds[first_ddp:], "expected SyncBN collectives between bucket launches"
