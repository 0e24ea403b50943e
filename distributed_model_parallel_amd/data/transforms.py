"""Minimal image transforms (torchvision is not installed).

Covers the reference's pipelines: CIFAR-10 ``RandomCrop(32, padding=4) +
RandomHorizontalFlip + ToTensor + Normalize`` (``model_parallel.py:77-87``)
and the ImageNet-style ``RandomResizedCrop / Resize + CenterCrop``.  Inputs
are PIL images or uint8 HWC numpy arrays; ``ToTensor`` yields float CHW in
[0, 1].  The GPU-side alternative (crop/flip/normalise/cast/layout in one HIP
kernel) is :func:`..data.gpu_augment.gpu_augment`.
"""
from __future__ import annotations

import math
import random
from typing import Callable, List, Sequence, Tuple

import numpy as np
import torch

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2023, 0.1994, 0.2010)
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def _to_np(img) -> np.ndarray:
    if isinstance(img, np.ndarray):
        return img
    return np.asarray(img.convert("RGB"))


class Compose:
    def __init__(self, ts: Sequence[Callable]):
        self.ts = list(ts)

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class RandomCrop:
    def __init__(self, size: int, padding: int = 0):
        self.size, self.padding = size, padding

    def __call__(self, img):
        a = _to_np(img)
        if self.padding:
            p = self.padding
            a = np.pad(a, ((p, p), (p, p), (0, 0)))
        h, w = a.shape[:2]
        i = random.randint(0, h - self.size)
        j = random.randint(0, w - self.size)
        return a[i:i + self.size, j:j + self.size]


class CenterCrop:
    def __init__(self, size: int):
        self.size = size

    def __call__(self, img):
        a = _to_np(img)
        h, w = a.shape[:2]
        i, j = (h - self.size) // 2, (w - self.size) // 2
        return a[i:i + self.size, j:j + self.size]


class Resize:
    """Resize the shorter side to `size` (PIL bilinear)."""

    def __init__(self, size: int):
        self.size = size

    def __call__(self, img):
        from PIL import Image
        im = img if not isinstance(img, np.ndarray) else Image.fromarray(img)
        w, h = im.size
        s = self.size / min(w, h)
        return np.asarray(im.convert("RGB").resize((max(1, round(w * s)), max(1, round(h * s))),
                                                   Image.BILINEAR))


class RandomResizedCrop:
    def __init__(self, size: int, scale=(0.08, 1.0), ratio=(3 / 4, 4 / 3)):
        self.size, self.scale, self.ratio = size, scale, ratio

    def __call__(self, img):
        from PIL import Image
        im = img if not isinstance(img, np.ndarray) else Image.fromarray(img)
        w, h = im.size
        area = w * h
        for _ in range(10):
            ta = area * random.uniform(*self.scale)
            ar = math.exp(random.uniform(math.log(self.ratio[0]), math.log(self.ratio[1])))
            cw, ch = int(round(math.sqrt(ta * ar))), int(round(math.sqrt(ta / ar)))
            if 0 < cw <= w and 0 < ch <= h:
                x0, y0 = random.randint(0, w - cw), random.randint(0, h - ch)
                break
        else:
            cw = ch = min(w, h)
            x0, y0 = (w - cw) // 2, (h - ch) // 2
        return np.asarray(im.convert("RGB").crop((x0, y0, x0 + cw, y0 + ch))
                          .resize((self.size, self.size), Image.BILINEAR))


class RandomHorizontalFlip:
    def __init__(self, p: float = 0.5):
        self.p = p

    def __call__(self, img):
        a = _to_np(img)
        return a[:, ::-1] if random.random() < self.p else a


class ToTensor:
    def __call__(self, img) -> torch.Tensor:
        a = np.ascontiguousarray(_to_np(img))
        return torch.from_numpy(a).permute(2, 0, 1).float().div_(255.0)


class ToUint8:
    """HWC uint8 tensor (for the GPU augmentation path: decode on CPU only)."""

    def __call__(self, img) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(_to_np(img)))


class Normalize:
    def __init__(self, mean: Sequence[float], std: Sequence[float]):
        self.mean = torch.tensor(mean).view(-1, 1, 1)
        self.std = torch.tensor(std).view(-1, 1, 1)

    def __call__(self, t: torch.Tensor) -> torch.Tensor:
        return (t - self.mean) / self.std


def cifar_train_transform():
    return Compose([RandomCrop(32, padding=4), RandomHorizontalFlip(), ToTensor(),
                    Normalize(CIFAR_MEAN, CIFAR_STD)])


def cifar_test_transform():
    return Compose([ToTensor(), Normalize(CIFAR_MEAN, CIFAR_STD)])


def imagenet_train_transform(size: int = 224):
    return Compose([RandomResizedCrop(size), RandomHorizontalFlip(), ToTensor(),
                    Normalize(IMAGENET_MEAN, IMAGENET_STD)])


def imagenet_val_transform(size: int = 224):
    return Compose([Resize(int(size * 256 / 224)), CenterCrop(size), ToTensor(),
                    Normalize(IMAGENET_MEAN, IMAGENET_STD)])
