"""The two multi-rank design risks VERDICT r5 (item 6) asked to close on the CPU.

(a) Precision of the bf16 bucket average.  The reducer averages bf16 buckets
    with ncclAvg in bf16 (csrc/ddp/reducer.cpp): RCCL's ring pre-scales every
    rank's input by 1/N (exact for N = 2, 4, 8) and rounds the partial sum to
    bf16 after each of the N - 1 reduce-scatter hops.  Measured here:
    * an exact emulation of that ring at N = 8 on gradient-like data bounds
      the relative RMS error of the average against fp64, next to the
      one-rounding floor (the fp64 average rounded to bf16 once);
    * an 8-rank gloo world running our DDP on a bf16 model: the reducer's
      averaged gradients against the fp64 average of every rank's local
      gradient, with the default bf16 reduction and with
      ``reduce_dtype=torch.float32`` (an fp32 copy of each bucket is reduced:
      one rounding, at the floor).
    Upstream DDP also reduces in the gradient dtype; the fp32 option exists
    for runs where the ~N-hop error matters.

(b) Two communicators on two streams (DDP buckets on the reducer's side stream,
    SyncBatchNorm moments on the compute stream) are deadlock-free only if every
    rank created them -- and so their streams, which the runtime maps onto
    hardware queues in creation order -- identically.  comm/rccl.py
    ``verify_comm_layout`` asserts that collectively at DDP and SyncBN
    communicator creation; here it passes on identical layouts and raises on
    every rank when one rank created an extra communicator first.
"""
import torch

from tests.dist_utils import run_world

BF16_EPS = 2.0 ** -8  # bf16 unit roundoff is 2^-9; one ulp at 1.0 is 2^-8


def _grads_like(n_ranks: int, numel: int, seed: int = 0) -> torch.Tensor:
    """Per-rank gradients: a shared signal plus per-rank noise of comparable
    size, with per-'layer' scales spread over 4 decades (as real grads are)."""
    g = torch.Generator().manual_seed(seed)
    scale = 10.0 ** (-4 * torch.rand(numel // 256, 1, generator=g)).expand(-1, 256).reshape(-1)
    signal = torch.randn(numel, generator=g, dtype=torch.float64)
    noise = torch.randn(n_ranks, numel, generator=g, dtype=torch.float64)
    return ((signal + noise) * scale).to(torch.bfloat16)


def _ring_avg_bf16(x: torch.Tensor) -> torch.Tensor:
    """RCCL's bf16 ring all-reduce with ncclAvg: inputs pre-scaled by 1/N, the
    partial sum rounded to bf16 after every hop (chunk c starts at rank c + 1)."""
    n, m = x.shape
    pre = (x.double() / n).to(torch.bfloat16)
    out = torch.empty(m, dtype=torch.bfloat16)
    chunks = torch.arange(m).chunk(n)
    for c, idx in enumerate(chunks):
        order = [(c + 1 + k) % n for k in range(n)]
        acc = pre[order[0], idx].float()
        for r in order[1:]:
            acc = (acc + pre[r, idx].float()).to(torch.bfloat16).float()
        out[idx] = acc.to(torch.bfloat16)
    return out


def _rel_rms(a: torch.Tensor, ref: torch.Tensor) -> float:
    return float((a.double() - ref).norm() / ref.norm())


def test_bf16_ring_average_error_is_bounded_at_8_ranks():
    x = _grads_like(8, 1 << 16)
    exact = x.double().mean(0)
    floor = _rel_rms(exact.to(torch.bfloat16), exact)  # one rounding of the exact average
    ring = _rel_rms(_ring_avg_bf16(x), exact)
    # measured: floor 1.63e-3, ring 3.15e-3 (1.9x: 7 hops, but the partial sums
    # of mixed sign partly cancel; the gloo world below: 1.71e-3 / 3.64e-3).  A bound a few times the floor, far below the per-rank
    # gradient noise the average is taken over (relative ~1 here).
    assert floor < 2e-3, floor
    assert floor < ring < 6 * floor, (ring, floor)
    assert ring < 4 * BF16_EPS, ring


def _ddp_avg_worker(rank, world, fp32):
    import torch.distributed as dist
    import torch.nn as nn
    from distributed_model_parallel_amd.parallel.distributed import DistributedDataParallel
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(64, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(),
                          nn.Linear(256, 10)).to(torch.bfloat16)
    local = nn.Sequential(nn.Linear(64, 256), nn.Tanh(), nn.Linear(256, 256), nn.Tanh(),
                          nn.Linear(256, 10)).to(torch.bfloat16)
    local.load_state_dict(model.state_dict())
    ddp = DistributedDataParallel(model, bucket_cap_mb=0.05, first_bucket_mb=0.01,
                                  reduce_dtype=torch.float32 if fp32 else None)
    torch.manual_seed(1000 + rank)
    x = torch.randn(32, 64).to(torch.bfloat16)
    ddp(x).float().pow(2).mean().backward()
    local(x).float().pow(2).mean().backward()
    mine = torch.cat([p.grad.reshape(-1) for p in local.parameters()]).double()
    got = torch.cat([p.grad.reshape(-1) for p in model.parameters()]).double()
    allg = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(allg, mine)
    exact = torch.stack(allg).mean(0)
    return {"err": _rel_rms(got, exact), "floor": _rel_rms(exact.to(torch.bfloat16), exact),
            "buckets": len(ddp.reducer.buckets())}


def test_ddp_bf16_bucket_average_gloo_8_ranks():
    res = run_world(_ddp_avg_worker, 8, False)
    assert all(r["buckets"] >= 2 for r in res), res
    for r in res:
        assert r["err"] < 6 * r["floor"] and r["err"] < 4 * BF16_EPS, r
    res32 = run_world(_ddp_avg_worker, 8, True)
    for r in res32:
        # fp32 reduction, rounded once into the bf16 bucket: at the floor
        assert r["err"] <= 1.05 * r["floor"] + 1e-12, r


def _layout_worker(rank, world, skew):
    import torch.distributed as dist
    from distributed_model_parallel_amd.comm.rccl import Communicator, verify_comm_layout
    dev = torch.device("cpu")
    if skew and rank == 1:
        Communicator(dev, purpose="extra")
    Communicator(dev, purpose="ddp")
    Communicator(dev, purpose="syncbn")
    try:
        dig = verify_comm_layout("test")
        return {"ok": True, "dig": dig}
    except RuntimeError as e:
        dist.barrier()
        return {"ok": False, "msg": str(e)}


def test_comm_layout_verified_collectively():
    same = run_world(_layout_worker, 2, False)
    assert all(r["ok"] for r in same) and same[0]["dig"] == same[1]["dig"] != 0, same
    skew = run_world(_layout_worker, 2, True)
    assert not any(r["ok"] for r in skew), skew
    assert all("communicator layout differs" in r["msg"] for r in skew), skew
