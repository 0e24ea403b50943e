"""Whole-model TRAIN-mode gradient parity of the native ResNet-50 step (VERDICT
r4 item 3): batch-statistics BN, the BN fold, the fused BN-backward
epilogues, the stride-phase data gradients and every other route the
headline bench takes, against stock PyTorch fp32 on the same weights and the
same input.

Regime: 224 px, batch 128, residual branches tamed (each bottleneck's last BN
gamma x 0.1; test_gpu_checkpointing.py uses 0.25) -- a random-init ResNet-50
at small batches is chaotic in bf16 (profiles/README.md finding 4).

What bf16 itself costs is measured, not assumed (tools/parity_probe.py,
profiles/parity_r5.md): STOCK PyTorch in bf16 lands at a per-parameter
gradient cosine of 0.971 median / 0.947 min from fp32 in this regime (0.90 /
0.83 at gamma 0.25, batch 64; 0.19 at gamma 1), while fp32 vs fp32 with the
input moved by one ulp stays at 0.99999.  So the bound is relative: the
native bf16 step must be at least as close to fp32 as stock bf16 is (the
native kernels measured 0.974 / 0.953, whole-model cosine 0.995), and a
second native run must agree with the first (0.99 median: the BN moments'
cross-block fp64 atomics land in run-dependent order at this batch)."""
import copy
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

pytestmark = pytest.mark.gpu

BATCH, SIZE, GAMMA, NCLS = 128, 224, 0.1, 100


@pytest.fixture(scope="module")
def runs():
    import parity_probe as pp
    from distributed_model_parallel_amd.utils import routes
    m0 = pp.build(GAMMA, NCLS)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(BATCH, 3, SIZE, SIZE, generator=g).bfloat16().float().cuda()
    y = torch.randint(0, NCLS, (BATCH,), generator=g).cuda()
    r0 = routes.route_counts()
    ln, gn = pp.grads_native(m0, x, y)
    trained = routes.active(routes.diff(routes.route_counts(), r0))
    ln2, gn2 = pp.grads_native(m0, x, y)
    l32, g32 = pp.grads_stock(m0, x, y)
    l16, g16 = pp.grads_stock(m0, x, y, torch.bfloat16)
    out = dict(native=(ln, gn), native2=(ln2, gn2), fp32=(l32, g32), bf16=(l16, g16), routes=trained, pp=pp)
    yield out
    torch.cuda.empty_cache()


def test_native_train_gradients_match_fp32(runs):
    pp = runs["pp"]
    ln, gn = runs["native"]
    l32, g32 = runs["fp32"]
    c = pp.compare(gn, g32)
    floor = pp.compare(runs["bf16"][1], g32)  # what bf16 itself costs, stock kernels
    print("native vs fp32", c, "stock bf16 vs fp32", floor)
    assert c["median"] >= floor["median"] - 0.005, (c, floor)
    assert c["p05"] >= floor["p05"] - 0.01, (c, floor)
    assert c["min"] >= floor["min"] - 0.02, (c, floor)
    assert c["conv_median"] >= floor["conv_median"] - 0.005, (c, floor)
    assert c["whole"] >= 0.99 and c["whole"] >= floor["whole"] - 0.002, (c, floor)
    assert abs(ln - l32) <= 1e-3 * abs(l32), (ln, l32)


def test_native_train_runs_are_consistent(runs):
    pp = runs["pp"]
    c = pp.compare(runs["native"][1], runs["native2"][1])
    print("native vs native", c)
    assert c["median"] >= 0.98 and c["min"] >= 0.95 and c["whole"] >= 0.995, c


def test_parity_run_takes_the_bench_routes(runs):
    """The routes of the headline step that this batch-64 run can take: the
    fold with and without the downsample, fused BN backward, halo and xl
    convolutions, stride-phase data gradients, ping-pong TN weight gradients."""
    need = {"bn_fold.fold", "bn_fold.fold_ds", "bn_fold.fold_fused_bwd", "conv1x1.fused_bn_bwd",
            "conv1x1.tn_xl", "conv_igemm.halo_fwd", "conv_igemm.halo_dgrad", "conv_igemm.halo_wgrad",
            "conv_igemm.xl_fwd", "conv_igemm.xl_dgrad", "conv_igemm.xl_dgrad_s2", "stem.halo",
            "fused.bn_relu_maxpool", "fused.stem_bn_relu_maxpool", "batchnorm.fused_bwd_moments"}
    from distributed_model_parallel_amd.utils import routes
    miss = routes.missing(need, runs["routes"])
    assert not miss, miss
