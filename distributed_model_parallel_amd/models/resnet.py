"""ResNet-18/34/50/101/152 (ImageNet layout, torchvision-compatible parameter
shapes and counts: ResNet-18 = 11,689,512, ResNet-50 = 25,557,032).

The BASELINE.json north-star workloads (ResNet-18 DP plumbing, ResNet-50 DDP /
DP / SyncBN) -- torchvision is not installed, so the models are our own.
MI355X-first choices:
  * every BN+ReLU and the bottleneck's BN+residual-add+ReLU run as ONE fused
    channels-last kernel (:class:`~..ops.batchnorm.BatchNormAct2d`), i.e. the
    residual add and both activations cost no extra HBM pass;
  * meant to run in ``torch.channels_last`` so convolutions and BN see NHWC;
  * ``zero_init_residual`` as in the usual large-batch recipe.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Type, Union

import torch
import torch.nn as nn

from ..ops.batchnorm import BatchNormAct2d
from ..ops.bn_fold import conv1x1_bn_fold, foldable, foldable_downsample
from ..ops.conv1x1 import Conv1x1
from ..ops.conv_igemm import ConvIG2d
from ..ops.fused import GradSlot, bn_relu_conv1x1, conv_bn, conv_bn_maxpool, grad_tap
from ..ops.pool import MaxPool2d, global_avg_pool
from ..ops.stem import StemConv2d


# bn2 -> conv3 prologue fusion (ops/fused.py bn_relu_conv1x1).  Off by default:
# measured on MI355X (profiles/README.md finding 6) the per-element BN+ReLU in
# the GEMM operand staging costs more (+0.2 ms forward GEMM, +0.5 ms weight
# gradient) than the removed BN apply pass saves (0.39 ms).  Kept as an API
# option (set_fuse_bn2_conv3; tests/test_gpu_models.py), not an env switch.
_FUSE_BN2_CONV3 = False


def set_fuse_bn2_conv3(on: bool) -> None:
    global _FUSE_BN2_CONV3
    _FUSE_BN2_CONV3 = bool(on)


def _conv3x3(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    # implicit-GEMM MFMA conv on MI355X (channels-last bf16, Cin % 64 == 0), BN moments fused
    return ConvIG2d(cin, cout, 3, stride=stride, padding=1)


def _conv1x1(cin: int, cout: int, stride: int = 1) -> nn.Conv2d:
    # MFMA GEMM on MI355X (channels-last bf16) with BN moments fused in its epilogue
    return Conv1x1(cin, cout, stride)


def _shortcut(ds: Optional[nn.Module], x: torch.Tensor) -> torch.Tensor:
    if ds is None:
        return x
    if isinstance(ds, nn.Sequential) and len(ds) == 2:
        return conv_bn(ds[0], ds[1], x)
    return ds(x)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = _conv3x3(cin, planes, stride)
        self.bn1 = BatchNormAct2d(planes, act="relu")
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = BatchNormAct2d(planes, act="relu")  # fused: relu(bn2(x) + identity)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        identity = _shortcut(self.downsample, x)
        out = conv_bn(self.conv1, self.bn1, x)
        return conv_bn(self.conv2, self.bn2, out, identity)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = _conv1x1(cin, planes)
        self.bn1 = BatchNormAct2d(planes, act="relu")
        self.conv2 = _conv3x3(planes, planes, stride)  # stride on the 3x3 (ResNet v1.5)
        self.bn2 = BatchNormAct2d(planes, act="relu")
        self.conv3 = _conv1x1(planes, planes * 4)
        self.bn3 = BatchNormAct2d(planes * 4, act="relu")  # fused residual add + relu
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        # x feeds conv1 and the shortcut: conv1's data-gradient GEMM absorbs the
        # shortcut's gradient (ops/fused.py GradSlot) instead of an add kernel.
        # The shortcut is built AFTER conv1 so its backward nodes run first.
        slot = GradSlot() if (self.training and torch.is_grad_enabled()) else None
        out = conv_bn(self.conv1, self.bn1, x, grad_slot=slot)
        xt = grad_tap(x, slot)
        fold = (self.training and not _FUSE_BN2_CONV3 and foldable(self.conv3, self.bn3, out)
                and isinstance(self.bn2, BatchNormAct2d))
        # the downsample conv + BN join the same folded GEMM (ops/bn_fold.py): its
        # output and the residual tensor are never materialised either
        fold_ds = fold and self.downsample is not None and foldable_downsample(
            self.downsample, xt, self.conv3.weight.shape[0])
        identity = None if fold_ds else _shortcut(self.downsample, xt)
        if _FUSE_BN2_CONV3 and self.training and isinstance(self.bn3, BatchNormAct2d) \
                and hasattr(self.conv2, "forward_with_moments"):
            # bn2's apply + ReLU runs inside conv3's GEMM (never materialised)
            raw, sums2 = self.conv2.forward_with_moments(out)
            out, sums3 = bn_relu_conv1x1(self.bn2, self.conv3, raw, sums2)
            return self.bn3(out, identity, sums=sums3)
        if fold:
            # bn3 folded through conv3 (ops/bn_fold.py): conv3's 4x-wide output is
            # never materialised; bn2's apply pass also reduces colsum(a2)
            if hasattr(self.conv2, "forward_with_moments"):
                raw, sums2 = self.conv2.forward_with_moments(out)
            else:
                raw, sums2 = self.conv2(out), None
            a2, asums = self.bn2(raw, sums=sums2, out_moments=True)
            if fold_ds:
                return conv1x1_bn_fold(self.conv3, self.bn3, a2, asums, downsample=self.downsample, x=xt)
            return conv1x1_bn_fold(self.conv3, self.bn3, a2, asums, identity)
        out = conv_bn(self.conv2, self.bn2, out)
        return conv_bn(self.conv3, self.bn3, out, identity)


class ResNet(nn.Module):
    def __init__(self, block: Type[Union[BasicBlock, Bottleneck]], layers: Sequence[int],
                 num_classes: int = 1000, zero_init_residual: bool = False,
                 stem_channels: int = 64):
        super().__init__()
        self.inplanes = stem_channels
        # 7x7/s2 stem as a space-to-depth MFMA implicit GEMM with fused BN moments
        self.conv1 = StemConv2d(3, stem_channels)
        self.bn1 = BatchNormAct2d(stem_channels, act="relu")
        self.maxpool = MaxPool2d(3, stride=2, padding=1)  # NHWC kernel, byte argmax
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                BatchNormAct2d(planes * block.expansion, act=None),
            )
        mods: List[nn.Module] = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            mods.append(block(self.inplanes, planes))
        return nn.Sequential(*mods)

    def forward_features(self, x: torch.Tensor) -> torch.Tensor:
        # stem: BN + ReLU applied inside the max pool (ops/fused.py conv_bn_maxpool)
        x = conv_bn_maxpool(self.conv1, self.bn1, self.maxpool, x)
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return global_avg_pool(x)  # channels-last broadcast backward (ops/pool.py)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.fc(self.forward_features(x))

    def as_sequential(self) -> nn.Sequential:
        """Atoms for the pipeline partitioner: stem, every block, head."""
        atoms: List[nn.Module] = [nn.Sequential(self.conv1, self.bn1, self.maxpool)]
        for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
            atoms.extend(list(layer))
        atoms.append(nn.Sequential(self.avgpool, nn.Flatten(1), self.fc))
        return nn.Sequential(*atoms)


def resnet18(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def resnet34(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def resnet50(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def resnet101(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def resnet152(num_classes: int = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)
