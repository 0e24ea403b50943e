"""Pipeline model-parallel oracle: an N-stage P2P
pipeline must produce the same loss and per-stage parameter gradients as the
sequential model in one process -- for any world size (reference defect 2),
every schedule, and the reference's ring loss placement."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from distributed_model_parallel_amd.parallel.pipeline import atom_costs, balanced_partition
from tests.dist_utils import run_world


def _mlp_atoms():
    torch.manual_seed(0)
    return nn.Sequential(nn.Sequential(nn.Flatten(), nn.Linear(48, 32), nn.ReLU()),
                         nn.Sequential(nn.Linear(32, 32), nn.Tanh()),
                         nn.Sequential(nn.Linear(32, 32), nn.ReLU()),
                         nn.Sequential(nn.Linear(32, 24), nn.ReLU()),
                         nn.Linear(24, 7))


def _mnv2_atoms():
    from distributed_model_parallel_amd.models import MobileNetV2
    torch.manual_seed(0)
    return MobileNetV2(num_classes=10).as_sequential()


def _data(kind, batch):
    g = torch.Generator().manual_seed(5)
    if kind == "mlp":
        return torch.randn(batch, 3, 4, 4, generator=g), torch.randint(0, 7, (batch,), generator=g)
    return torch.randn(batch, 3, 32, 32, generator=g), torch.randint(0, 10, (batch,), generator=g)


def _sequential_grads(kind, batch, micro):
    # the workers run single-threaded; match the CPU kernels' reduction order
    nt = torch.get_num_threads()
    torch.set_num_threads(1)
    try:
        atoms = _mlp_atoms() if kind == "mlp" else _mnv2_atoms()
        x, y = _data(kind, batch)
        total = 0.0
        for xs, ys in zip(torch.chunk(x, micro), torch.chunk(y, micro)):
            loss = F.cross_entropy(atoms(xs), ys) / micro
            loss.backward()
            total += float(loss.detach())
        return total, [[p.grad.clone() for p in a.parameters()] for a in atoms]
    finally:
        torch.set_num_threads(nt)


def _pipe_worker(rank, world, kind, batch, micro, schedule, loss_on):
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mlp_atoms() if kind == "mlp" else _mnv2_atoms()
    shape = (3, 4, 4) if kind == "mlp" else (3, 32, 32)
    comm = Communicator(torch.device("cpu"))
    pipe = Pipeline(atoms, comm, shape, micro_batches=micro, schedule=schedule, loss_on=loss_on)
    x, y = _data(kind, batch)
    res = pipe.train_step(x if rank == 0 else None, y if rank == 0 else None)
    lo, hi = pipe.partition[rank]
    grads = {i: [p.grad.clone() for p in atoms[i].parameters()] for i in range(lo, hi)}
    ev = pipe.eval_step(x if rank == 0 else None, y if rank == 0 else None)
    return {"loss": res.loss, "grads": grads, "partition": pipe.partition, "eval": ev.loss,
            "top1": res.top1}


@pytest.mark.parametrize("world,schedule,micro,loss_on", [
    (2, "naive", 1, "last"), (3, "gpipe", 4, "last"), (4, "1f1b", 4, "last"),
    (2, "1f1b", 6, "last"), (3, "gpipe", 2, "first"), (4, "naive", 1, "first")])
def test_pipeline_mlp_matches_sequential(world, schedule, micro, loss_on):
    batch = 12
    ref_loss, ref_grads = _sequential_grads("mlp", batch, micro)
    res = run_world(_pipe_worker, world, "mlp", batch, micro, schedule, loss_on)
    assert res[0]["loss"] == pytest.approx(ref_loss, rel=1e-5, abs=1e-6)
    for r in res:
        for i, gs in r["grads"].items():
            for g, rg in zip(gs, ref_grads[i]):
                torch.testing.assert_close(g, rg, atol=1e-6, rtol=1e-5)
    assert res[0]["eval"] is not None


@pytest.mark.parametrize("world", [2, 3, 4])
def test_pipeline_mobilenetv2_any_world_size(world):
    """The reference's MobileNetV2 pipeline, at world sizes it could not run (2, 3)."""
    batch = 4
    ref_loss, ref_grads = _sequential_grads("mnv2", batch, 1)
    res = run_world(_pipe_worker, world, "mnv2", batch, 1, "naive", "last")
    assert res[0]["loss"] == pytest.approx(ref_loss, rel=1e-4)
    for r in res:
        for i, gs in r["grads"].items():
            for g, rg in zip(gs, ref_grads[i]):
                torch.testing.assert_close(g, rg, atol=1e-4, rtol=1e-3)
    covered = sorted(i for r in res for i in r["grads"])
    assert covered == list(range(len(ref_grads)))


def test_balanced_partition_properties():
    costs = [5, 1, 1, 1, 1, 1, 5, 2, 2]
    for k in range(1, len(costs) + 1):
        parts = balanced_partition(costs, k)
        assert len(parts) == k and parts[0][0] == 0 and parts[-1][1] == len(costs)
        assert all(a < b for a, b in parts)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(k - 1))
    assert max(sum(costs[a:b]) for a, b in balanced_partition(costs, 3)) == 8  # brute-force optimum


def test_atom_costs_mobilenet():
    atoms = _mnv2_atoms()
    c = atom_costs(atoms, torch.zeros(2, 3, 32, 32))
    assert len(c) == 20 and all(v > 0 for v in c)


def _ragged_worker(rank, world, partition):
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mnv2_atoms() if partition == "reference" else _mlp_atoms()
    shape = (3, 32, 32) if partition == "reference" else (3, 4, 4)
    kind = "mnv2" if partition == "reference" else "mlp"
    comm = Communicator(torch.device("cpu"))
    pipe = Pipeline(atoms, comm, shape, micro_batches=4, schedule="gpipe", partition=partition)
    x, y = _data(kind, 12)
    pipe.train_step(x if rank == 0 else None, y if rank == 0 else None)
    for p in atoms.parameters():
        p.grad = None
    x, y = _data(kind, 7)           # dynamic last batch: 7 rows over 4 micro-batches
    res = pipe.train_step(x if rank == 0 else None, y if rank == 0 else None)
    lo, hi = pipe.partition[rank]
    return {"loss": res.loss, "partition": pipe.partition,
            "grads": {i: [p.grad.clone() for p in atoms[i].parameters()] for i in range(lo, hi)}}


@pytest.mark.parametrize("world,partition", [(3, None), (4, "reference")])
def test_pipeline_dynamic_last_batch(world, partition):
    """A smaller final batch after a full one (SURVEY §4.2 pipeline oracle) -- and the
    reference's own 4-way MobileNetV2 cut."""
    kind = "mnv2" if partition == "reference" else "mlp"
    ref_loss, ref_grads = _sequential_grads(kind, 7, 4)
    res = run_world(_ragged_worker, world, partition)
    if partition == "reference":
        assert res[0]["partition"] == [(0, 4), (4, 10), (10, 16), (16, 20)]
    assert res[0]["loss"] == pytest.approx(ref_loss, rel=1e-4, abs=1e-6)
    for r in res:
        for i, gs in r["grads"].items():
            for g, rg in zip(gs, ref_grads[i]):
                torch.testing.assert_close(g, rg, atol=1e-4, rtol=1e-3)


def _static_batch_worker(rank, world):
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mlp_atoms()
    comm = Communicator(torch.device("cpu"))
    pipe = Pipeline(atoms, comm, (3, 4, 4), micro_batches=2, schedule="1f1b", static_batch=6)
    x, y = _data("mlp", 6)
    r1 = pipe.train_step(x if rank == 0 else None, y if rank == 0 else None)  # static: no size message
    # a ragged batch must be passed explicitly on every rank
    r2 = pipe.train_step(x[:5] if rank == 0 else None, y[:5] if rank == 0 else None, batch_size=5)
    err = None
    if rank == 0:
        try:
            pipe._batch_size(x[:4])
        except ValueError as e:
            err = str(e)
    return {"l1": r1.loss if r1.valid else None, "l2": r2.loss if r2.valid else None, "err": err}


def test_pipeline_static_batch_contract():
    """the batch size is part of the static contract (no
    per-step message / host sync); rank 0 refuses a batch that breaks it."""
    res = run_world(_static_batch_worker, 2)
    assert res[0]["l1"] is not None and res[0]["l2"] is not None
    assert abs(res[1]["l1"] - res[0]["l1"]) < 1e-6  # the last stage holds the same loss
    assert "contract is 6" in res[0]["err"]


def test_batch_schedule_matches_loader_and_rejects_ragged_batches():
    """the CLI checks the static batch contract against the
    loader's batch sampler before the loop (every rank then stops together)."""
    import pytest
    from torch.utils.data import BatchSampler, DataLoader, SequentialSampler, TensorDataset
    from distributed_model_parallel_amd.train.cli import batch_schedule
    ds = TensorDataset(torch.zeros(50, 2))
    assert batch_schedule(DataLoader(ds, batch_size=16), 16) == (4, 2)
    assert batch_schedule(DataLoader(ds, batch_size=16, drop_last=True), 16) == (3, 16)
    assert batch_schedule(DataLoader(ds, batch_size=10), 10) == (5, 10)
    with pytest.raises(ValueError):
        batch_schedule(DataLoader(ds, batch_size=8), 16)

    class Ragged:  # a custom batch sampler that breaks the contract mid-epoch
        def __iter__(self):
            return iter([list(range(16)), list(range(16, 28)), list(range(28, 44))])

        def __len__(self):
            return 3
    with pytest.raises(ValueError):
        batch_schedule(DataLoader(ds, batch_sampler=Ragged()), 16)
    ok = BatchSampler(SequentialSampler(range(40)), 16, False)
    assert batch_schedule(DataLoader(ds, batch_sampler=list(ok)), 16) == (3, 8)


def _bad_batch_worker(rank, world):
    import time
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mlp_atoms()
    pipe = Pipeline(atoms, Communicator(torch.device("cpu")), (3, 4, 4), micro_batches=2,
                    schedule="1f1b", static_batch=6)
    x, y = _data("mlp", 5)  # breaks the static contract of 6
    if rank == 0:
        try:
            pipe.train_step(x, y)
        except ValueError:
            time.sleep(30)  # stay alive (a notebook, a caught error): peers must not rely on our exit
            raise SystemExit(7)
        raise SystemExit(0)
    pipe.train_step(None, None)  # blocks in a receive that rank 0 never sends
    raise SystemExit(0)


def test_pipeline_contract_violation_exits_every_rank():
    """a bad batch on rank 0 used to leave every later stage
    blocked in a receive forever.  Rank 0 now publishes the failure through the
    store (utils/debug.FailureBroadcast) and the other stages exit non-zero
    while rank 0 is still alive."""
    from tests.dist_utils import run_world_exitcodes
    codes = run_world_exitcodes(_bad_batch_worker, 3, timeout_s=25)
    assert codes[1] == 3 and codes[2] == 3, codes   # peers: failure flag seen, os._exit(3)


def _graphed_worker(rank, world, micro):
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mlp_atoms()
    comm = Communicator(torch.device("cpu"))
    pipe = Pipeline(atoms, comm, (3, 4, 4), micro_batches=micro, schedule="1f1b", graphs=True, static_batch=12)
    x, y = _data("mlp", 12)
    res = []
    for _ in range(2):  # the second step reuses the slots
        for p in atoms.parameters():
            p.grad = None if p.grad is None else p.grad.zero_()
        res.append(pipe.train_step(x if rank == 0 else None, y if rank == 0 else None))
    lo, hi = pipe.partition[rank]
    grads = {i: [p.grad.clone() for p in atoms[i].parameters()] for i in range(lo, hi)}
    depth = next(iter(pipe._graphs.values())).depth
    return {"loss": [r.loss for r in res] if rank == 0 else None, "grads": grads, "depth": depth}


@pytest.mark.parametrize("world,micro", [(2, 4), (3, 6), (4, 4), (4, 2)])
def test_pipeline_graphed_slot_schedule_matches_sequential(world, micro):
    """The slot schedule of Pipeline(graphs=True) (1F1B on static per-slot
    buffers, at most S - r micro-batches in flight on stage r) on the CPU
    stand-ins of the captured graphs: same loss and per-stage gradients as the
    sequential model, twice in a row (slots reused across steps)."""
    ref_loss, ref_grads = _sequential_grads("mlp", 12, micro)
    res = run_world(_graphed_worker, world, micro)
    for loss in res[0]["loss"]:
        assert loss == pytest.approx(ref_loss, rel=1e-5, abs=1e-6)
    for r, out in enumerate(res):
        assert out["depth"] == min(micro, world - r)
        for i, gs in out["grads"].items():
            for g, rg in zip(gs, ref_grads[i]):
                torch.testing.assert_close(g, rg, atol=1e-6, rtol=1e-5)


def _recapture_worker(rank, world):
    import warnings
    from distributed_model_parallel_amd.comm.rccl import Communicator
    from distributed_model_parallel_amd.parallel.pipeline import Pipeline
    atoms = _mlp_atoms()
    comm = Communicator(torch.device("cpu"))
    pipe = Pipeline(atoms, comm, (3, 4, 4), micro_batches=4, schedule="1f1b", graphs=True, static_batch=12)
    x, y = _data("mlp", 12)
    with warnings.catch_warnings(record=True) as caught:
        warnings.simplefilter("always")
        for step in range(4):
            for p in atoms.parameters():
                p.grad = None  # a stock optimizer's zero_grad(set_to_none=True): storage moves
            pipe.train_step(x if rank == 0 else None, y if rank == 0 else None)
    return {"recaptures": pipe.recaptures,
            "warned": sum("re-captured again" in str(w.message) for w in caught)}


def test_pipeline_graph_recaptures_are_counted_and_warned():
    """a re-capture forced by moved gradient storage must not be
    silent -- counted on the pipeline and warned about once it repeats."""
    for r in run_world(_recapture_worker, 2):
        assert r["recaptures"] == 3 and r["warned"] == 1, r
