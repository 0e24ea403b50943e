"""Pipeline engine and its RCCL point-to-point transport on one MI355X
(the pipeline had only ever run on gloo).

With one GPU the stages cannot be on different ranks, so this covers what one
rank can: the engine at world size 1 on device (bf16, channels-last, every
schedule, fused cross-entropy, stats returned without a host sync), and the
RCCL send/recv path itself as a grouped self-exchange through the native
communicator (the same ncclSend/ncclRecv pair every pipeline hop issues).
"""

import pytest
import torch
import torch.distributed as dist
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _pg():
    import torch.distributed as dist
    if not dist.is_initialized():  # one rank: an in-process store, no TCP port to race for
        dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)


@pytest.fixture(scope="module", autouse=True)
def _destroy_pg():
    yield
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def _comm():
    _pg()
    from distributed_model_parallel_amd.comm.rccl import Communicator
    return Communicator(torch.device("cuda", 0))


def test_rccl_grouped_self_p2p_roundtrip():
    comm = _comm()
    assert comm.native is not None
    x = torch.randn(64, 24, 32, 32, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    buf = torch.empty_like(x)
    comm.batch_p2p([(x, 0, True), (buf, 0, False)])
    comm.wait()
    assert torch.equal(buf, x)


@pytest.mark.parametrize("schedule,micro", [("naive", 1), ("gpipe", 4), ("1f1b", 4)])
def test_pipeline_world1_on_gpu_matches_sequential(schedule, micro):
    from distributed_model_parallel_amd.models import MobileNetV2
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    comm = _comm()
    torch.manual_seed(0)
    atoms = MobileNetV2(num_classes=10).as_sequential()
    pipe = Pipeline(atoms, comm, (3, 32, 32), micro_batches=micro, schedule=schedule,
                    device=torch.device("cuda", 0), dtype=torch.float32, static_batch=32)
    x = torch.randn(32, 3, 32, 32)
    y = torch.randint(0, 10, (32,))
    r = pipe.train_step(x, y)
    assert r.valid and r.loss_tensor.is_cuda  # device stats, no host sync yet
    grads = [p.grad.clone() for p in pipe.module.parameters()]
    # oracle: the same stage module, micro-batched by hand, stock cross-entropy
    for p in pipe.module.parameters():
        p.grad = None
    total = 0.0
    for xs, ys in zip(torch.chunk(x.cuda(), micro), torch.chunk(y.cuda(), micro)):
        loss = F.cross_entropy(pipe.module(xs).float(), ys) / micro
        loss.backward()
        total += float(loss.detach())
    assert abs(r.loss - total) < 1e-3 * max(1.0, abs(total))
    # MIOpen's fp32 weight gradients accumulate in a run-dependent order, and the
    # bias gradients of BNs feeding another BN cancel to ~0 (two identical stock
    # runs differ O(1) there, relative): compare per tensor in norm with an
    # absolute floor at the model's gradient scale.  An engine bug -- a lost or
    # doubled micro-batch -- is O(1) of the tensor's own norm.
    norms = sorted(float(p.grad.norm()) for p in pipe.module.parameters())
    floor = 1e-3 * norms[len(norms) // 2]
    for a, p in zip(grads, pipe.module.parameters()):
        err = float((a - p.grad).norm())
        assert err <= 1e-2 * float(p.grad.norm()) + floor, (err, float(p.grad.norm()), floor)


def test_pipeline_world1_bf16_trains():
    from distributed_model_parallel_amd.models import MobileNetV2
    from distributed_model_parallel_amd.ops.optim import MasterSGD
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    comm = _comm()
    torch.manual_seed(0)
    pipe = Pipeline(MobileNetV2(num_classes=10).as_sequential(), comm, (3, 32, 32), micro_batches=4,
                    schedule="1f1b", device=torch.device("cuda", 0), dtype=torch.bfloat16, channels_last=True,
                    static_batch=64)
    opt = MasterSGD(pipe.module.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(64, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (64,), generator=g)
    losses = []
    for _ in range(30):  # memorise one batch
        r = pipe.train_step(x, y)
        opt.step()
        opt.zero_grad()
        losses.append(r.loss_tensor)
    first, last = float(losses[0]), float(losses[-1])
    assert last < 0.5 * first, (first, last)


@pytest.mark.parametrize("dtype,cl", [(torch.float32, False), (torch.bfloat16, True)])
def test_pipeline_graphed_stage_matches_eager(dtype, cl):
    """Pipeline(graphs=True): the 1F1B micro-batches replay
    captured stage graphs.  Against the eager engine on the same weights over
    three steps with MasterSGD updates between them (the replays must read the
    updated weights and accumulate the micro-batch gradients in place): same
    losses and gradients; running statistics updated once per micro-batch."""
    import copy
    from distributed_model_parallel_amd.models import MobileNetV2
    from distributed_model_parallel_amd.ops.optim import MasterSGD
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    comm = _comm()
    torch.manual_seed(0)
    atoms = MobileNetV2(num_classes=10).as_sequential()
    pipes, opts = [], []
    for graphs in (False, True):
        p = Pipeline(copy.deepcopy(atoms), comm, (3, 32, 32), micro_batches=4, schedule="1f1b",
                     device=torch.device("cuda", 0), dtype=dtype, channels_last=cl, static_batch=64,
                     graphs=graphs)
        pipes.append(p)
        opts.append(MasterSGD(p.module.parameters(), lr=0.05, momentum=0.9))
    g = torch.Generator().manual_seed(1)
    tol = 2e-3 if dtype == torch.float32 else 3e-2
    for step in range(3):
        x = torch.randn(64, 3, 32, 32, generator=g)
        y = torch.randint(0, 10, (64,), generator=g)
        res = [p.train_step(x, y) for p in pipes]
        # fp32 stages run library convolutions, which are not replay-safe: eager
        assert bool(pipes[1]._graphs) == (dtype == torch.bfloat16), "graphed path taken / not taken"
        la, lb = float(res[0].loss), float(res[1].loss)
        if dtype == torch.bfloat16 or step == 0:
            assert abs(la - lb) <= tol * max(1.0, abs(la)), (step, la, lb)
            assert abs(res[0].top1 - res[1].top1) <= 100.0 / 64 * 2, step
        num = den = 0.0
        for pa, pb in zip(pipes[0].module.parameters(), pipes[1].module.parameters()):
            num += float((pa.grad.float() - pb.grad.float()).pow(2).sum())
            den += float(pa.grad.float().pow(2).sum())
        rel = (num / den) ** 0.5
        # fp32 (both engines eager): MIOpen's fp32 weight gradients differ run to
        # run in the last bits (1.7e-3 at step 0, round 5) and BN over 16-image
        # micro-batches amplifies that after an SGD step (0.30 at step 1) --
        # compare fp32 at step 0 only
        if dtype == torch.bfloat16 or step == 0:
            assert rel < (1e-2 if dtype == torch.float32 else 5e-2), (step, rel)
        for o in opts:
            o.step()
            o.zero_grad()
    for (n, a), b in zip(pipes[0].module.named_buffers(), pipes[1].module.buffers()):
        if a.dtype.is_floating_point:
            if dtype == torch.bfloat16:
                torch.testing.assert_close(b.float(), a.float(), atol=tol * 10, rtol=tol * 10, msg=n)
        else:
            assert torch.equal(a, b), n  # 3 steps x 4 micro-batches, not more (warm-up undone)
