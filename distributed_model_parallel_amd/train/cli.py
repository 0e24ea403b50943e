"""Training CLI: data parallel (DDP / single-process DP) and pipeline model
parallel, flag-compatible with the reference scripts.

Reference entry points (§5.6):
  ``python model_parallel.py DIR --world-size 4 --dist-url tcp://127.0.0.1:1224
  --dist-backend nccl --lr 0.4 --epochs 90 -type Imagenet -b 512 -j 12 --wd 1e-4
  --momentum 0.9`` and ``python data_parallel.py --lr 0.4 [-r]``.

Equivalents here::

  torchrun --nproc-per-node 8 -m distributed_model_parallel_amd.train.cli DIR \\
      --parallel ddp --arch resnet50 -type Imagenet -b 256 --epochs 90
  python -m distributed_model_parallel_amd.train.cli --parallel dp --arch mobilenetv2 \\
      -type CIFAR10 DIR -b 512 -r
  python -m distributed_model_parallel_amd.train.cli --parallel pipe --world-size 4 \\
      --arch mobilenetv2 -type CIFAR10 DIR --micro-batches 8 --schedule 1f1b

``--synthetic`` (or no DIR) trains on synthetic data of the dataset's shape.
Honoured flags the reference parsed but ignored (defect 4): ``-b``, ``-j``,
``-type`` and ``DIR``.
"""
from __future__ import annotations

import argparse
import os
import sys
from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native data / model parallel training")
    p.add_argument("data", nargs="?", default="", metavar="DIR", help="dataset root (empty: synthetic)")
    p.add_argument("--dist-url", default=None, help="init method (default env:// from torchrun)")
    p.add_argument("--world-size", default=None, type=int,
                   help="processes to spawn for --parallel pipe without torchrun")
    p.add_argument("--dist-backend", default=None, help="nccl (=RCCL) on GPU, gloo on CPU")
    p.add_argument("--lr", "--learning-rate", default=0.4, type=float, dest="lr")
    p.add_argument("--epochs", default=90, type=int)
    p.add_argument("-type", "--dataset-type", default="CIFAR10", dest="dataset_type")
    p.add_argument("-b", "--batch-size", default=512, type=int,
                   help="per-process batch for ddp; total batch for dp and pipe")
    p.add_argument("-j", "--workers", default=4, type=int)
    p.add_argument("--wd", "--weight-decay", default=1e-4, type=float, dest="weight_decay")
    p.add_argument("--momentum", default=0.9, type=float)
    p.add_argument("-r", "--resume", action="store_true")
    p.add_argument("--arch", default="mobilenetv2")
    p.add_argument("--parallel", default="ddp", choices=["ddp", "dp", "pipe", "none"])
    p.add_argument("--bucket-cap-mb", default=25.0, type=float)
    p.add_argument("--dp-graphs", action="store_true",
                   help="--parallel dp: replicas' forward/backward as captured hipGraphs (no replica threads)")
    p.add_argument("--sync-bn", action="store_true")
    p.add_argument("--dtype", default="auto", choices=["auto", "fp32", "bf16"],
                   help="auto: bf16 (fp32 master weights) on GPU -- the native MFMA path -- fp32 on CPU")
    p.add_argument("--channels-last", dest="channels_last", action="store_true", default=None,
                   help="NHWC activations (default on GPU: every native conv/BN kernel is NHWC)")
    p.add_argument("--no-channels-last", dest="channels_last", action="store_false")
    p.add_argument("--synthetic", action="store_true")
    p.add_argument("--micro-batches", default=1, type=int)
    p.add_argument("--no-pipe-graphs", action="store_true",
                   help="--parallel pipe on GPU: eager micro-batches instead of captured stage graphs")
    p.add_argument("--schedule", default="1f1b", choices=["naive", "gpipe", "1f1b"])
    p.add_argument("--partition", default="balanced", choices=["balanced", "reference"],
                   help="pipeline stage cut: FLOP-balanced (any ws) or the reference's MobileNetV2 cut")
    p.add_argument("--warmup-epochs", default=10, type=int, help="linear lr warm-up (0 = none)")
    p.add_argument("--lr-steps", default="", metavar="E1,E2,...",
                   help="step decay at these epochs instead of cosine (reference no-BN study: 30,60)")
    p.add_argument("--lr-gamma", default=0.1, type=float, help="decay factor of --lr-steps")
    p.add_argument("--checkpoint-segments", default=0, type=int, metavar="K",
                   help="activation checkpointing: recompute the model in K segments in backward "
                        "(reference large-batch runs '2048(checkpoint)', Readme.md:168,192; 0 = off)")
    p.add_argument("--steps-per-epoch", default=0, type=int, help="cap iterations per epoch (0 = all)")
    p.add_argument("--log-dir", default="./log")
    p.add_argument("--checkpoint", default="./checkpoint/ckpt.pth")
    p.add_argument("--seed", default=0, type=int)
    p.add_argument("--watchdog", default=None, type=float, metavar="SECONDS",
                   help="abort (exit 1, so torchrun can restart) when the collective stream makes "
                        "no progress for SECONDS (default 1800 when distributed on GPU, 0 = off)")
    return p


def _datasets(args):
    from ..data import DatasetCollection, transforms as T
    cifar = args.dataset_type in ("CIFAR10", "SyntheticCIFAR")
    if args.synthetic or not args.data:
        kind = "SyntheticCIFAR" if cifar or args.arch.startswith("mobilenet") else "Synthetic"
        return DatasetCollection(kind, "").init()
    if cifar:
        tr, va = T.cifar_train_transform(), T.cifar_test_transform()
    else:
        tr, va = T.imagenet_train_transform(), T.imagenet_val_transform()
    return DatasetCollection(args.dataset_type, args.data, tr, va).init()


def _lr_steps(args):
    return [int(v) for v in args.lr_steps.split(",") if v.strip()] if args.lr_steps else None


def _num_classes(args) -> int:
    return {"CIFAR10": 10, "SyntheticCIFAR": 10, "CUB200": 200, "Place365": 365}.get(
        args.dataset_type, 10 if (args.synthetic or not args.data) and args.arch.startswith("mobilenet") else 1000)


# --------------------------------------------------------------------------- #
def run_data_parallel(args, env) -> None:
    from ..data import prepare_dataloaders
    from ..models import build_model
    from ..ops.optim import FlatSGD, MasterSGD
    from ..parallel.data_parallel import DataParallel
    from ..parallel.distributed import DistributedDataParallel
    from ..parallel.sync_batchnorm import SyncBatchNorm
    from ..utils.checkpoint import load_checkpoint, save_checkpoint
    from ..utils.logging import MetricsLogger
    from ..utils.metrics import AverageMeter, accuracy
    from ..utils.precision import cast_model, parse_dtype
    from ..ops.loss import cross_entropy
    from ..utils.profiling import trace_range
    from ..utils.schedule import build_schedule
    from ..utils.timers import StepTimer

    dev = env.device
    dtype = parse_dtype(args.dtype)
    model = build_model(args.arch, num_classes=_num_classes(args))
    if args.checkpoint_segments > 1:
        from ..utils.checkpointing import enable_activation_checkpointing
        enable_activation_checkpointing(model, args.checkpoint_segments)
    if args.sync_bn and args.parallel == "ddp":
        model = SyncBatchNorm.convert_sync_batchnorm(model)
    model = model.to(dev)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    if dtype != torch.float32:
        cast_model(model, dtype)
    if args.parallel == "ddp":
        net = DistributedDataParallel(model, bucket_cap_mb=args.bucket_cap_mb, flat_parameters=True)
        opt = FlatSGD(net, lr=args.lr, momentum=args.momentum, weight_decay=args.weight_decay)
    else:
        # fp32 master weights for bf16 models: same update as DDP's FlatSGD
        opt = MasterSGD(model.parameters(), lr=args.lr, momentum=args.momentum,
                        weight_decay=args.weight_decay)
        net = DataParallel(model, graphs=args.dp_graphs) if args.parallel == "dp" else model
    sched = build_schedule(opt, args.epochs, args.warmup_epochs, _lr_steps(args), args.lr_gamma)
    from ..utils.debug import rank0_first
    with rank0_first():  # defect 6: rank 0 prepares / indexes the dataset before the others read it
        train_ds, val_ds = _datasets(args)
    sampler, train_loader, val_loader = prepare_dataloaders(
        train_ds, val_ds, args.batch_size, args.workers, distributed=args.parallel == "ddp" and env.distributed,
        pin_memory=dev.type == "cuda", seed=args.seed)
    start_epoch, best = 0, 0.0
    if args.resume and os.path.exists(args.checkpoint):
        meta = load_checkpoint(args.checkpoint, net, opt, sched, map_location=dev)
        start_epoch, best = meta["epoch"] + 1, meta["acc"]
    logger = MetricsLogger(args.log_dir, f"{args.parallel}_{args.arch}", env.rank,
                           text_file=f"{args.parallel}_{args.batch_size}.txt")

    def to_dev(x, y):
        x = x.to(dev, dtype, non_blocking=True)
        if args.channels_last and x.dim() == 4:
            x = x.contiguous(memory_format=torch.channels_last)
        return x, y.to(dev, non_blocking=True)

    timer = StepTimer(dev)
    for epoch in range(start_epoch, args.epochs):
        if sampler is not None:
            sampler.set_epoch(epoch)
        net.train()
        lm, am = AverageMeter(), AverageMeter()
        it = iter(train_loader)
        i = 0
        while not (args.steps_per_epoch and i >= args.steps_per_epoch):
            with timer.region("data"):  # reference data_time (utils.py:48): host wait + H2D
                batch = next(it, None)
                if batch is None:
                    break
                x, y = to_dev(*batch)
            with timer.region("step"), trace_range("train.step"):
                out = net(x)
                loss = cross_entropy(out, y)
                loss.backward()
                opt.step()
                opt.zero_grad()
            lm.update(loss.detach(), y.shape[0])
            am.update(accuracy(out, y)[0], y.shape[0])
            i += 1
        if dev.type == "cuda":
            torch.cuda.synchronize()
        tm = timer.summary()  # device time of the step (HIP events), host time of the data wait
        step_s, data_s = tm.get("step", 0.0) / 1e3, tm.get("data_host", 0.0) / 1e3
        vl, va = evaluate(net, val_loader, to_dev, args)
        sched.step()
        if env.is_main and va > best:
            best = va
            save_checkpoint(args.checkpoint, net, opt, sched, epoch, best)
        logger.log(epoch, loss_train=lm.avg, acc1_train=am.avg, loss_val=vl, acc1_val=va,
                   time_per_batch=step_s + data_s, time_load_perbatch=data_s,
                   images_per_sec=(args.batch_size * max(1, env.world_size if args.parallel == "ddp" else 1))
                   / max(step_s + data_s, 1e-9), lr=opt.param_groups[0]["lr"])


@torch.no_grad()
def evaluate(net, loader, to_dev, args):
    from ..utils.metrics import AverageMeter, accuracy
    net.eval()
    lm, am = AverageMeter(), AverageMeter()
    for i, (x, y) in enumerate(loader):
        if args.steps_per_epoch and i >= args.steps_per_epoch:
            break
        x, y = to_dev(x, y)
        out = net(x)
        lm.update(F.cross_entropy(out.float(), y), y.shape[0])
        am.update(accuracy(out, y)[0], y.shape[0])
    return lm.avg, am.avg


# --------------------------------------------------------------------------- #
def batch_schedule(loader, batch_size: int):
    """(number of batches, size of the last) of `loader`, read from its batch
    sampler without loading data; ValueError unless every batch but the last
    has `batch_size` samples (the pipeline's static shape contract)."""
    bsamp = getattr(loader, "batch_sampler", None)
    sampler = getattr(bsamp, "sampler", None)
    if bsamp is not None and type(bsamp) is torch.utils.data.BatchSampler and sampler is not None:
        n_items, bs, drop = len(sampler), bsamp.batch_size, bsamp.drop_last
        if bs != batch_size:
            raise ValueError(f"loader batch size {bs} != contract {batch_size}")
        n = n_items // bs if drop else -(-n_items // bs)
        last = bs if (drop or n_items % bs == 0) else n_items % bs
    else:  # a custom batch sampler: walk its index lists (no data is loaded)
        sizes = [len(b) for b in (bsamp if bsamp is not None else [])]
        if not sizes:
            raise ValueError("loader has no inspectable batch sampler")
        if any(s != batch_size for s in sizes[:-1]) or sizes[-1] > batch_size:
            raise ValueError(f"batch sizes {sorted(set(sizes))} do not follow the contract {batch_size}")
        n, last = len(sizes), sizes[-1]
    if n != len(loader):
        raise ValueError(f"batch sampler yields {n} batches, len(loader) = {len(loader)}")
    return n, last


def run_pipeline(args, env) -> None:
    from ..comm.rccl import Communicator
    from ..data import prepare_dataloaders
    from ..models import INPUT_SHAPES, build_model
    from ..ops.optim import MasterSGD
    from ..parallel.pipeline import Pipeline
    from ..utils.checkpoint import save_checkpoint, stage_checkpoint_path
    from ..utils.logging import MetricsLogger
    from ..utils.precision import parse_dtype
    from ..utils.profiling import trace_range
    from ..utils.schedule import build_schedule
    from ..utils.timers import StepTimer

    torch.manual_seed(args.seed)  # every rank builds the same full model (reference: unseeded)
    model = build_model(args.arch, num_classes=_num_classes(args))
    (c, h, w), _ = INPUT_SHAPES.get(args.arch, ((3, 32, 32), 10))
    comm = Communicator(env.device)
    pipe = Pipeline(model.as_sequential(), comm, (c, h, w), micro_batches=args.micro_batches,
                    schedule=args.schedule, dtype=parse_dtype(args.dtype),
                    channels_last=args.channels_last, partition=args.partition,
                    # one GPU only (see train/step.py): multi-rank GPU pipelines run eagerly
                    graphs=env.device.type == "cuda" and not args.no_pipe_graphs and comm.size == 1)
    opt = MasterSGD(pipe.module.parameters(), lr=args.lr, momentum=args.momentum,
                    weight_decay=args.weight_decay)
    sched = build_schedule(opt, args.epochs, args.warmup_epochs, _lr_steps(args), args.lr_gamma)
    logger = MetricsLogger(args.log_dir, f"pipe_{args.arch}", env.rank, text_file=f"{args.batch_size}.txt")
    if env.rank == 0:
        train_ds, val_ds = _datasets(args)
        _, train_loader, val_loader = prepare_dataloaders(train_ds, val_ds, args.batch_size, args.workers,
                                                          pin_memory=env.device.type == "cuda")
        vbs = val_loader.batch_size or args.batch_size
        # the static batch contract of every step, checked against the loaders'
        # batch samplers BEFORE the loop: a mismatch found later would raise on
        # rank 0 only while the other stages wait in a receive
        bad = ""
        try:
            n_train, last_t = batch_schedule(train_loader, args.batch_size)
            n_val, last_v = batch_schedule(val_loader, vbs)
        except ValueError as e:
            bad, n_train = str(e), -1
            n_val = last_t = last_v = 0
    else:
        train_loader = val_loader = None
        n_train = n_val = last_t = last_v = vbs = 0
    # only rank 0 loads data; the others learn the iteration counts and batch
    # sizes once (defect 6), so no step needs a batch-size message or host sync
    counts = torch.tensor([n_train, n_val, last_t, last_v, vbs], dtype=torch.int64, device=env.device)
    comm.broadcast(counts, 0)
    comm.synchronize()
    n_train, n_val, last_t, last_v, vbs = (int(v) for v in counts.tolist())
    if n_train < 0:  # every rank stops here, together
        raise ValueError("pipeline: the data loader's batches do not follow the static batch contract"
                         + (f" ({bad})" if env.rank == 0 else " (see rank 0)"))
    n_train_all, n_val_all = n_train, n_val
    if args.steps_per_epoch:
        n_train, n_val = min(n_train, args.steps_per_epoch), min(n_val, args.steps_per_epoch)
    timer = StepTimer(env.device)
    for epoch in range(args.epochs):
        it = iter(train_loader) if train_loader is not None else None
        sums = []  # per-step device stats, read once per epoch
        for i in range(n_train):
            with timer.region("data"):
                x, y = next(it) if it is not None else (None, None)
            bs = last_t if i == n_train_all - 1 else args.batch_size
            with timer.region("step"), trace_range("pipe.train_step"):
                r = pipe.train_step(x, y, batch_size=bs)
                opt.step()
                opt.zero_grad()
            if r.valid:
                sums.append(r)
        loss_s = sum(r.loss for r in sums)
        acc_s = sum(r.top1 for r in sums)
        tm = timer.summary()
        tot_t = (tm.get("step", 0.0) + tm.get("data_host", 0.0)) / 1e3 * max(n_train, 1)
        tot_d = tm.get("data_host", 0.0) / 1e3 * max(n_train, 1)
        vit = iter(val_loader) if val_loader is not None else None
        vl, va = 0.0, 0.0
        for i in range(n_val):
            x, y = next(vit) if vit is not None else (None, None)
            r = pipe.eval_step(x, y, batch_size=last_v if i == n_val_all - 1 else vbs)
            if r.valid:
                vl += r.loss
                va += r.top1
        sched.step()
        save_checkpoint(stage_checkpoint_path(args.checkpoint, env.rank), pipe.module, opt, sched, epoch,
                        all_ranks=True)
        if env.rank == 0:
            logger.log(epoch, loss_train=loss_s / max(n_train, 1), acc1_train=acc_s / max(n_train, 1),
                       loss_val=vl / max(n_val, 1), acc1_val=va / max(n_val, 1),
                       time_per_batch=tot_t / max(n_train, 1), time_load_perbatch=tot_d / max(n_train, 1))


def _spawn_entry(rank: int, world: int, args) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      LOCAL_WORLD_SIZE=str(world))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    main_worker(args)


def main_worker(args) -> None:
    from ..utils.env import destroy_distributed, init_distributed, seed_everything
    from ..utils import miopen_db
    env = init_distributed(backend=args.dist_backend, dist_url=args.dist_url)
    gpu = env.device.type == "cuda"
    if args.dtype == "auto":
        args.dtype = "bf16" if gpu else "fp32"
    if args.channels_last is None:
        args.channels_last = gpu
    if env.device.type == "cuda":
        miopen_db.seed("use")  # committed MIOpen find db (skips the first-step solver search)
    seed_everything(args.seed + (env.rank if args.parallel == "ddp" else 0))
    dog = start_watchdog(args.watchdog, env)
    try:
        if args.parallel == "pipe":
            run_pipeline(args, env)
        else:
            run_data_parallel(args, env)
    finally:
        if dog is not None:
            dog.stop()
        destroy_distributed()


def start_watchdog(seconds: Optional[float], env):
    """Start a CommWatchdog on the process's communicator: a
    collective stream stuck for `seconds` ends the process with exit code 1
    (no re-exec), so torchrun --max-restarts can restart the job."""
    if seconds is None:
        seconds = 1800.0 if (env.distributed and env.device.type == "cuda") else 0.0
    if seconds <= 0 or env.device.type != "cuda":
        return None
    from ..comm.rccl import default_communicator
    from ..utils.debug import CommWatchdog
    return CommWatchdog(default_communicator(env.device), timeout_s=seconds,
                        interval_s=min(5.0, seconds / 4)).start()


def main(argv: Optional[list] = None) -> int:
    args = build_parser().parse_args(argv)
    if args.parallel == "pipe" and args.world_size and "RANK" not in os.environ:
        import torch.multiprocessing as mp
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        mp.spawn(_spawn_entry, args=(args.world_size, args), nprocs=args.world_size, join=True)
        return 0
    main_worker(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
