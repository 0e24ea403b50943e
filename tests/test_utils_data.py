"""Unit tests: accuracy, schedules, checkpoint round trip, logging, datasets,
transforms, model shapes/param counts (SURVEY.md §4 layer 1)."""
import json
import os

import numpy as np
import pytest
import torch

from distributed_model_parallel_amd.models import (MobileNetV2, build_model, mobilenet_v2_nobn, resnet18,
                                                   resnet50, vit_b_16)
from distributed_model_parallel_amd.utils.metrics import AverageMeter, accuracy
from distributed_model_parallel_amd.utils.schedule import LinearWarmup, WarmupCosine, cosine_lr


def test_param_counts_match_reference_and_torchvision():
    assert sum(p.numel() for p in MobileNetV2().parameters()) == 2_296_922
    assert sum(p.numel() for p in resnet18().parameters()) == 11_689_512
    assert sum(p.numel() for p in resnet50().parameters()) == 25_557_032
    assert sum(p.numel() for p in vit_b_16().parameters()) == 86_567_656
    assert len(list(resnet50().parameters())) == 161


def test_mobilenet_partition_shapes():
    """Stage boundary shapes of the reference's 4-way cut."""
    m = MobileNetV2().eval()
    atoms = m.as_sequential()
    x = torch.randn(2, 3, 32, 32)
    outs = []
    with torch.no_grad():
        for a in atoms:
            x = a(x)
            outs.append(tuple(x.shape))
    assert min(x.min() for x in [atoms[0](torch.randn(2, 3, 32, 32))]) >= 0  # stem keeps its ReLU (defect 3)
    assert outs[3] == (2, 24, 32, 32)    # stem + blocks 0..2 (reference rank 0 output)
    assert outs[9] == (2, 64, 8, 8)      # + blocks 3..8 (rank 1)
    assert outs[15] == (2, 160, 4, 4)    # + blocks 9..14 (rank 2)
    assert outs[-1] == (2, 10)


def test_nobn_has_no_batchnorm():
    m = mobilenet_v2_nobn()
    assert not any(isinstance(x, torch.nn.BatchNorm2d) for x in m.modules())
    assert m(torch.randn(2, 3, 32, 32)).shape == (2, 10)


def test_accuracy_hand_computed():
    out = torch.tensor([[0.1, 0.9, 0.0], [0.8, 0.1, 0.1], [0.2, 0.3, 0.5], [0.5, 0.4, 0.1]])
    tgt = torch.tensor([1, 1, 2, 1])
    a1, a2 = accuracy(out, tgt, topk=(1, 2))
    assert a1.item() == pytest.approx(50.0)
    assert a2.item() == pytest.approx(100.0)
    m = AverageMeter()
    m.update(a1, 4)
    m.update(100.0, 4)
    assert m.avg == pytest.approx(75.0)


def test_warmup_cosine_schedule():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=0.4)
    s = WarmupCosine(opt, epochs=90, warmup_epochs=10)
    lrs = [opt.param_groups[0]["lr"]]
    for e in range(1, 90):
        s.step()
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs[0] == pytest.approx(0.4 * cosine_lr(1, 0, 90) / 10)
    assert lrs[9] == pytest.approx(0.4 * cosine_lr(1, 9, 90))
    assert lrs[-1] < 1e-3 and max(lrs) <= 0.4


def test_linear_warmup_dampening_context():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.SGD([p], lr=1.0)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda e: 1.0)
    w = LinearWarmup(opt, warmup_period=4)
    assert opt.param_groups[0]["lr"] == pytest.approx(0.25)
    for k in range(2, 6):
        with w.dampening():
            sched.step()
        assert opt.param_groups[0]["lr"] == pytest.approx(min(1.0, k / 4))


def test_checkpoint_roundtrip(tmp_path):
    from distributed_model_parallel_amd.utils.checkpoint import load_checkpoint, save_checkpoint
    m = resnet18(num_classes=10)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    m(torch.randn(2, 3, 32, 32)).sum().backward()
    opt.step()
    s = WarmupCosine(opt, 10, 2)
    s.step()
    path = str(tmp_path / "ck" / "ckpt.pth")
    save_checkpoint(path, torch.nn.DataParallel(m), opt, s, epoch=3, best_acc=55.5)
    m2 = resnet18(num_classes=10)
    opt2 = torch.optim.SGD(m2.parameters(), lr=0.1, momentum=0.9)
    s2 = WarmupCosine(opt2, 10, 2)
    meta = load_checkpoint(path, m2, opt2, s2)
    assert meta["epoch"] == 3 and meta["acc"] == 55.5
    for a, b in zip(m.state_dict().values(), m2.state_dict().values()):
        torch.testing.assert_close(a, b)
    assert s2.epoch == 1
    # safe loader reads it; wrapped models keep the reference's module. prefix
    raw = torch.load(path, weights_only=True)
    assert all(k.startswith("module.") for k in raw["net"])
    # reference-format dict with module. prefix loads too
    ref = {"net": {"module." + k: v for k, v in m.state_dict().items()}, "acc": 1.0, "epoch": 7}
    torch.save(ref, tmp_path / "ref.pth")
    assert load_checkpoint(str(tmp_path / "ref.pth"), resnet18(num_classes=10))["epoch"] == 7


def test_metrics_logger_creates_dirs(tmp_path):
    from distributed_model_parallel_amd.utils.logging import MetricsLogger
    d = tmp_path / "does" / "not" / "exist"
    lg = MetricsLogger(str(d), "mp", rank=0, text_file="512.txt", echo=False)
    lg.log(0, loss_train=1.5, acc1_train=10.0, loss_val=1.2, acc1_val=20.0, time_per_batch=0.1)
    text = (d / "512.txt").read_text()
    assert "step:0  loss_train:1.5  acc1_train:10.0  loss_val:1.2  acc1_val:20.0  time_per_batch:0.1" in text
    rec = json.loads((d / "mp.rank0.jsonl").read_text().splitlines()[0])
    assert rec["loss_train"] == 1.5


def test_cifar_binary_and_transforms(tmp_path):
    from distributed_model_parallel_amd.data import CIFAR10, DatasetCollection, transforms as T
    d = tmp_path / "cifar-10-batches-bin"
    d.mkdir()
    rng = np.random.default_rng(0)
    for name in [f"data_batch_{i}" for i in range(1, 6)] + ["test_batch"]:
        recs = np.concatenate([rng.integers(0, 10, (7, 1)), rng.integers(0, 256, (7, 3072))], 1)
        recs.astype(np.uint8).tofile(d / f"{name}.bin")
    tr, va = DatasetCollection("CIFAR10", str(tmp_path), T.cifar_train_transform(),
                               T.cifar_test_transform()).init()
    assert len(tr) == 35 and len(va) == 7
    x, y = tr[3]
    assert x.shape == (3, 32, 32) and 0 <= y < 10
    raw = CIFAR10(str(tmp_path), train=False)
    assert raw[0][0].shape == (32, 32, 3)


def test_cub_and_imagefolder(tmp_path):
    from PIL import Image

    from distributed_model_parallel_amd.data import DatasetCollection, transforms as T
    base = tmp_path / "CUB_200_2011"
    (base / "images" / "001.a").mkdir(parents=True)
    for i in range(1, 5):
        Image.new("RGB", (40, 30), (i * 10, 0, 0)).save(base / "images" / "001.a" / f"{i}.jpg")
    (base / "images.txt").write_text("".join(f"{i} 001.a/{i}.jpg\n" for i in range(1, 5)))
    (base / "image_class_labels.txt").write_text("".join(f"{i} {1 + i % 2}\n" for i in range(1, 5)))
    (base / "train_test_split.txt").write_text("1 1\n2 0\n3 1\n4 0\n")
    tf = T.Compose([T.CenterCrop(24), T.ToTensor()])
    tr, va = DatasetCollection("CUB200", str(tmp_path), tf, tf).init()
    assert len(tr) == 2 and len(va) == 2
    assert {tr[0][1], tr[1][1]} <= {0, 1}
    for split in ("train", "val"):
        for c in ("cat", "dog"):
            (tmp_path / "inet" / split / c).mkdir(parents=True)
            Image.new("RGB", (64, 48)).save(tmp_path / "inet" / split / c / "x.png")
    tr, va = DatasetCollection("Imagenet", str(tmp_path / "inet"), T.imagenet_train_transform(32),
                               T.imagenet_val_transform(32)).init()
    assert len(tr) == 2 and tr[1][0].shape == (3, 32, 32) and tr.classes == ["cat", "dog"]
    with pytest.raises(ValueError):
        DatasetCollection("nope", str(tmp_path)).init()


def test_build_model_registry():
    assert build_model("resnet18", num_classes=3)(torch.randn(1, 3, 64, 64)).shape == (1, 3)
    with pytest.raises(ValueError):
        build_model("vgg")


def test_reference_partition_matches_reference_cut():
    from distributed_model_parallel_amd.parallel.pipeline import reference_partition
    # model_parallel.py:101-104 at ws=4: rank0 conv1/bn1/layers[0:3], rank1 layers[3:9],
    # rank2 layers[9:15], rank3 layers[15:] + head + linear  (atoms: stem=0, block i = i+1)
    assert reference_partition(20, 4) == [(0, 4), (4, 10), (10, 16), (16, 20)]
    assert reference_partition(20, 2) == [(0, 4), (4, 20)]
    assert reference_partition(20, 3) == [(0, 4), (4, 10), (10, 20)]
