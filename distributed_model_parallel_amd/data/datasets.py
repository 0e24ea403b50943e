"""Datasets: the reference's ``DatasetCollection`` factory (ImageNet folder,
CUB-200-2011, CIFAR-10, Places365-small; ``dataset/dataset_collection.py:8-69``,
SURVEY C13-C15) without torchvision/pandas, plus synthetic datasets for
benchmarking (no network access: BASELINE.json mandates synthetic data).

Fixes vs the reference: unknown types raise instead of returning None;
Places365 "val" reads the validation list (defect 10); nothing downloads, and
:func:`prepare_dataloaders` adds a ``DistributedSampler`` for DDP and avoids
building loaders on ranks that never read data (defect 6).  CIFAR-10 is read
from the binary release (``cifar-10-batches-bin``) or the python release
through a restricted unpickler that only materialises plain containers and
numpy arrays.
"""
from __future__ import annotations

import io
import os
import pickle
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

IMG_EXTS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


def pil_loader(path: str):
    from PIL import Image
    with open(path, "rb") as f:
        return Image.open(f).convert("RGB")


# --------------------------------------------------------------------------- #
class SyntheticImages(Dataset):
    """Deterministic random images/labels (shape of ImageNet or CIFAR)."""

    def __init__(self, length: int, shape=(3, 224, 224), num_classes: int = 1000, seed: int = 0,
                 dtype=torch.float32):
        self.length, self.shape, self.num_classes, self.seed, self.dtype = length, tuple(shape), num_classes, seed, dtype

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        return (torch.randn(self.shape, generator=g).to(self.dtype),
                int(torch.randint(0, self.num_classes, (1,), generator=g)))


class ImageFolder(Dataset):
    """root/<class>/<image> layout (ImageNet train/ and val/)."""

    def __init__(self, root: str, transform: Optional[Callable] = None, loader=pil_loader):
        self.root = root
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        if not classes:
            raise FileNotFoundError(f"no class folders under {root}")
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        self.samples: List[Tuple[str, int]] = []
        for c in classes:
            for dp, _, fs in sorted(os.walk(os.path.join(root, c))):
                for f in sorted(fs):
                    if f.lower().endswith(IMG_EXTS):
                        self.samples.append((os.path.join(dp, f), self.class_to_idx[c]))
        self.classes = classes
        self.transform = transform
        self.loader = loader

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        p, t = self.samples[i]
        img = self.loader(p)
        return (self.transform(img) if self.transform else img), t


class CUB200(Dataset):
    """CUB-200-2011: images.txt, image_class_labels.txt, train_test_split.txt;
    labels shifted to 0-based (reference ``CUBDataset`` :8-27, :48-61)."""

    base_folder = "CUB_200_2011/images"

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None,
                 loader=pil_loader):
        base = os.path.join(root, "CUB_200_2011")

        def read(name):
            with open(os.path.join(base, name)) as f:
                return dict(line.split() for line in f if line.strip())

        paths = read("images.txt")
        labels = read("image_class_labels.txt")
        split = read("train_test_split.txt")
        want = "1" if train else "0"
        self.samples = [(paths[k], int(labels[k]) - 1) for k in sorted(paths, key=int) if split[k] == want]
        self.root, self.transform, self.loader = root, transform, loader

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        p, t = self.samples[i]
        img = self.loader(os.path.join(self.root, self.base_folder, p))
        return (self.transform(img) if self.transform else img), t


class _SafeUnpickler(pickle.Unpickler):
    """Only plain containers and numpy array reconstruction (CIFAR python batches)."""

    ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy", "ndarray"), ("numpy", "dtype"), ("builtins", "bytes")}

    def find_class(self, module, name):
        if (module, name) in self.ALLOWED:
            import importlib
            return getattr(importlib.import_module(module), name)
        raise pickle.UnpicklingError(f"blocked global {module}.{name}")


class CIFAR10(Dataset):
    """CIFAR-10 from ``cifar-10-batches-bin`` (preferred) or ``cifar-10-batches-py``."""

    def __init__(self, root: str, train: bool = True, transform: Optional[Callable] = None):
        self.transform = transform
        binp = os.path.join(root, "cifar-10-batches-bin")
        pyp = os.path.join(root, "cifar-10-batches-py")
        names = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
        xs, ys = [], []
        if os.path.isdir(binp):
            for n in names:
                raw = np.fromfile(os.path.join(binp, n + ".bin"), dtype=np.uint8).reshape(-1, 3073)
                ys.append(raw[:, 0].astype(np.int64))
                xs.append(raw[:, 1:].reshape(-1, 3, 32, 32))
        elif os.path.isdir(pyp):
            for n in names:
                with open(os.path.join(pyp, n), "rb") as f:
                    d = _SafeUnpickler(f, encoding="bytes").load()
                xs.append(np.asarray(d[b"data"], dtype=np.uint8).reshape(-1, 3, 32, 32))
                ys.append(np.asarray(d[b"labels"], dtype=np.int64))
        else:
            raise FileNotFoundError(f"no CIFAR-10 data under {root} (no network download)")
        self.data = np.concatenate(xs).transpose(0, 2, 3, 1)  # NHWC uint8
        self.targets = np.concatenate(ys)

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        img = self.data[i]
        return (self.transform(img) if self.transform else img), int(self.targets[i])


class Places365Small(Dataset):
    """Places365-standard small (256x256): data_256/ + places365_train_standard.txt,
    val_256/ + places365_val.txt."""

    def __init__(self, root: str, split: str = "train-standard", transform: Optional[Callable] = None,
                 loader=pil_loader):
        if split == "train-standard":
            lst, folder = "places365_train_standard.txt", "data_256"
        elif split == "val":
            lst, folder = "places365_val.txt", "val_256"
        else:
            raise ValueError(f"unsupported Places365 split {split!r}")
        with open(os.path.join(root, lst)) as f:
            rows = [l.split() for l in f if l.strip()]
        self.samples = [(os.path.join(root, folder, p.lstrip("/")), int(t)) for p, t in rows]
        self.transform, self.loader = transform, loader

    def __len__(self):
        return len(self.samples)

    def __getitem__(self, i):
        p, t = self.samples[i]
        img = self.loader(p)
        return (self.transform(img) if self.transform else img), t


class DatasetCollection:
    """Factory keyed by the reference's type strings: Imagenet, CUB200, CIFAR10,
    Place365 (plus Synthetic / SyntheticCIFAR)."""

    def __init__(self, type: str, path: str, compose_train=None, compose_val=None):
        self.type, self.path = type, path
        self.compose = {"train": compose_train, "val": compose_val}

    def init(self) -> Tuple[Dataset, Dataset]:
        t, p, c = self.type, self.path, self.compose
        if t == "Imagenet":
            return ImageFolder(os.path.join(p, "train"), c["train"]), ImageFolder(os.path.join(p, "val"), c["val"])
        if t == "CUB200":
            return CUB200(p, True, c["train"]), CUB200(p, False, c["val"])
        if t == "CIFAR10":
            return CIFAR10(p, True, c["train"]), CIFAR10(p, False, c["val"])
        if t == "Place365":
            return Places365Small(p, "train-standard", c["train"]), Places365Small(p, "val", c["val"])
        if t == "Synthetic":
            return SyntheticImages(1281, (3, 224, 224), 1000), SyntheticImages(500, (3, 224, 224), 1000, seed=1)
        if t == "SyntheticCIFAR":
            return SyntheticImages(5000, (3, 32, 32), 10), SyntheticImages(1000, (3, 32, 32), 10, seed=1)
        raise ValueError(f"unknown dataset type {t!r}")


def prepare_dataloaders(train_ds: Dataset, val_ds: Dataset, batch_size: int, workers: int,
                        distributed: bool = False, val_batch_size: Optional[int] = None,
                        pin_memory: bool = True, seed: int = 0):
    """Train/val loaders; a DistributedSampler shards the data under DDP (the
    reference's dead ``prepare_dataloader`` used sampler=None, ``utils.py:12-31``)."""
    sampler = None
    if distributed:
        sampler = torch.utils.data.distributed.DistributedSampler(train_ds, shuffle=True, seed=seed)
    train = DataLoader(train_ds, batch_size=batch_size, shuffle=sampler is None, sampler=sampler,
                       num_workers=workers, pin_memory=pin_memory, drop_last=False,
                       persistent_workers=workers > 0)
    val = DataLoader(val_ds, batch_size=val_batch_size or batch_size, shuffle=False,
                     num_workers=workers, pin_memory=pin_memory)
    return sampler, train, val
