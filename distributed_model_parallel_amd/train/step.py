"""One data-parallel training step, shared by bench.py, smoke() and the CLI.

Per step (DDP mode): forward of the local micro-batch (bf16, channels-last),
cross-entropy in fp32, backward with bucketed RCCL all-reduce overlapped by
the C++ reducer, one fused flat SGD launch per dtype group, one fill per
group to zero the gradient buckets.  Nothing is skipped or cached: every step
reads the input batch, runs the full model and updates every parameter.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..models import INPUT_SHAPES, build_model
from ..ops.loss import cross_entropy
from ..ops.optim import FlatSGD, MasterSGD
from ..utils.precision import cast_model


@dataclass
class StepConfig:
    model: str = "resnet50"
    batch_size: int = 256            # per GPU
    image_size: Optional[int] = None
    num_classes: Optional[int] = None
    dtype: torch.dtype = torch.bfloat16
    channels_last: bool = True
    parallel: str = "ddp"           # ddp | syncbn | dp | pipe | none
    bucket_cap_mb: float = 25.0
    first_bucket_mb: float = 1.0
    dp_devices: int = 1             # parallel == "dp": GPUs driven by the single process
    dp_replicas: int = 1            # parallel == "dp": replicas per GPU (>1 aliases several
                                    # replicas onto one device, so scatter / replicate /
                                    # parallel_apply / gather / reduce-add all run on 1 GPU)
    graph: bool = False             # capture the whole step in a hipGraph (constant LR, static data)
    lr: float = 0.1
    momentum: float = 0.9
    weight_decay: float = 1e-4
    seed: int = 0
    micro_batches: int = 8          # parallel == "pipe"
    schedule: str = "1f1b"          # parallel == "pipe": naive | gpipe | 1f1b
    partition: str = "balanced"     # parallel == "pipe": balanced | reference
    checkpoint_segments: int = 0    # activation checkpointing of the block trunk (0 = off)
    dp_graphs: bool = False         # parallel == "dp": replicas as captured hipGraphs (dp_graphs.py)
    pipe_graphs: bool = True        # parallel == "pipe" on GPU: 1F1B micro-batches on captured stage graphs
    extra: dict = field(default_factory=dict)


@dataclass
class TrainState:
    cfg: StepConfig
    model: nn.Module
    wrapped: nn.Module
    optimizer: torch.optim.Optimizer
    step: Callable[[], torch.Tensor]
    images: torch.Tensor
    labels: torch.Tensor


def synthetic_batch(cfg: StepConfig, device: torch.device, generator_seed: int = 1234,
                    batch: Optional[int] = None):
    (c, h, w), ncls = INPUT_SHAPES[cfg.model]
    if cfg.image_size:
        h = w = cfg.image_size
    ncls = cfg.num_classes or ncls
    b = batch or cfg.batch_size
    g = torch.Generator(device="cpu").manual_seed(generator_seed)
    x = torch.randn(b, c, h, w, generator=g).to(device=device, dtype=cfg.dtype)
    if cfg.channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, ncls, (b,), generator=g).to(device)
    return x, y


def build_train_state(cfg: StepConfig, device: torch.device) -> TrainState:
    if cfg.parallel == "pipe":
        return build_pipeline_state(cfg, device)
    if cfg.graph:
        if device.type != "cuda":
            raise ValueError("graph capture needs a GPU")
        # Build (and later warm up / capture) on ONE side stream: the DDP reducer
        # keeps the parameters' AccumulateGrad nodes alive, and a node created on
        # the default stream would sync against it inside the capture.
        side = torch.cuda.Stream(device=device)
        side.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(side):
            st = _build_train_state(cfg, device)
        from .graphed import GraphedStep
        # two eager calls, the capture on the third: bench.py's default
        # --warmup 3 then times replays only (with warmup=3 the capture landed
        # in the first timed step and inflated --graph rows by ~3 ms / 10 steps)
        st.step = GraphedStep(st.step, warmup=2, stream=side)
        return st
    return _build_train_state(cfg, device)


def _build_train_state(cfg: StepConfig, device: torch.device) -> TrainState:
    from ..parallel.distributed import DistributedDataParallel
    from ..parallel.sync_batchnorm import SyncBatchNorm

    torch.manual_seed(cfg.seed)
    kw = {}
    if cfg.num_classes:
        kw["num_classes"] = cfg.num_classes
    if cfg.image_size and cfg.model.startswith("vit"):
        kw["image_size"] = cfg.image_size
    model = build_model(cfg.model, **kw)
    if cfg.checkpoint_segments > 1:
        from ..utils.checkpointing import enable_activation_checkpointing
        enable_activation_checkpointing(model, cfg.checkpoint_segments)
    if cfg.parallel == "syncbn":
        model = SyncBatchNorm.convert_sync_batchnorm(model)
    model = model.to(device)
    if cfg.channels_last:
        model = model.to(memory_format=torch.channels_last)
    if cfg.dtype != torch.float32:
        cast_model(model, cfg.dtype)
    ndp = max(1, cfg.dp_devices) if (cfg.parallel == "dp" and device.type == "cuda") else 1
    # DP: the single process feeds batch_size images PER GPU (weak scaling, same
    # per-GPU work as DDP), scattered from device_ids[0]
    x, y = synthetic_batch(cfg, device, batch=cfg.batch_size * ndp)

    if cfg.parallel in ("ddp", "syncbn"):
        wrapped = DistributedDataParallel(model, bucket_cap_mb=cfg.bucket_cap_mb,
                                          first_bucket_mb=cfg.first_bucket_mb,
                                          flat_parameters=True)
        opt = FlatSGD(wrapped, lr=cfg.lr, momentum=cfg.momentum, weight_decay=cfg.weight_decay)

        def step() -> torch.Tensor:
            out = wrapped(x)
            loss = cross_entropy(out, y)
            loss.backward()
            opt.step()
            opt.zero_grad()
            return loss
    elif cfg.parallel == "dp":
        from ..parallel.data_parallel import DataParallel
        # fp32 master weights + momentum, one launch per dtype group (same update as DDP's FlatSGD)
        opt = MasterSGD(model.parameters(), lr=cfg.lr, momentum=cfg.momentum,
                        weight_decay=cfg.weight_decay)
        reps = max(1, cfg.dp_replicas)
        wrapped = DataParallel(model, device_ids=[d for d in range(ndp) for _ in range(reps)]
                               if device.type == "cuda" else None, graphs=cfg.dp_graphs)

        def step() -> torch.Tensor:
            out = wrapped(x)
            loss = cross_entropy(out, y)
            loss.backward()
            opt.step()
            opt.zero_grad()
            return loss
    else:
        wrapped = model
        opt = MasterSGD(model.parameters(), lr=cfg.lr, momentum=cfg.momentum,
                        weight_decay=cfg.weight_decay)

        def step() -> torch.Tensor:
            out = model(x)
            loss = cross_entropy(out, y)
            loss.backward()
            opt.step()
            opt.zero_grad()
            return loss

    return TrainState(cfg, model, wrapped, opt, step, x, y)


def build_pipeline_state(cfg: StepConfig, device: torch.device) -> TrainState:
    """Pipeline model parallelism across the process group (one stage per rank).

    ``cfg.batch_size`` is the WHOLE batch entering stage 0 (the reference's
    model-parallel run feeds 512 images per step through 4 stages,
    ``model_parallel.py:92``); it is cut into ``cfg.micro_batches`` micro-batches
    scheduled naive / gpipe / 1f1b.  Every stage updates its own slice with the
    same fp32-master SGD as the data-parallel paths.  ``step()`` returns the
    loss on rank 0 (and a zero tensor elsewhere).
    """
    from ..comm.rccl import default_communicator
    from ..parallel.pipeline import Pipeline

    torch.manual_seed(cfg.seed)  # every rank builds the same full model, keeps its stage
    kw = {"num_classes": cfg.num_classes} if cfg.num_classes else {}
    model = build_model(cfg.model, **kw)
    if not hasattr(model, "as_sequential"):
        raise ValueError(f"--parallel pipe needs a model with as_sequential() (got {cfg.model})")
    (c, h, w), _ = INPUT_SHAPES[cfg.model]
    if cfg.image_size:
        h = w = cfg.image_size
    comm = default_communicator(device)
    pipe = Pipeline(model.as_sequential(), comm, (c, h, w), micro_batches=cfg.micro_batches,
                    schedule=cfg.schedule, device=device, dtype=cfg.dtype,
                    channels_last=cfg.channels_last, partition=cfg.partition,
                    static_batch=cfg.batch_size,  # every rank knows it: no per-step size message
                    # captured stage slots on one GPU only: the multi-stage slot
                    # schedule is verified on the CPU stand-ins (tests/test_pipeline.py)
                    # but never with RCCL between captured stages (a 1-GPU box cannot
                    # host two RCCL ranks), so multi-rank GPU pipelines run eagerly
                    graphs=cfg.pipe_graphs and device.type == "cuda" and comm.size == 1)
    opt = MasterSGD(pipe.module.parameters(), lr=cfg.lr, momentum=cfg.momentum,
                    weight_decay=cfg.weight_decay)
    x, y = synthetic_batch(cfg, device) if pipe.is_first else (None, None)
    zero = torch.zeros((), device=device)

    def step() -> torch.Tensor:
        r = pipe.train_step(x, y)
        opt.step()
        opt.zero_grad()
        lt = r.loss_tensor if r.valid else None  # device tensor: no host sync per step
        return lt if lt is not None else zero

    return TrainState(cfg, pipe.module, pipe, opt, step, x, y)
