from .datasets import (CIFAR10, CUB200, DatasetCollection, ImageFolder, Places365Small, SyntheticImages,
                       prepare_dataloaders)
from . import transforms

__all__ = ["CIFAR10", "CUB200", "DatasetCollection", "ImageFolder", "Places365Small", "SyntheticImages",
           "prepare_dataloaders", "transforms"]
