"""ResNet family with the reference's module tree (`pytorch_model.py:14-113`).

State-dict keys and shapes are identical to the reference ``ResNet18(10)``
(122 keys, 11,173,962 params for CIFAR-10), so a checkpoint written by this
framework loads into the reference module and vice versa.  These eager
modules are the *definition* of the architecture: the native MI355X engine
(``mercury_amd.engine``) lowers them to its own NHWC/bf16 MFMA kernels and
shares their parameters through a flat buffer.

Differences from the reference:
  * ``ResNet101`` / ``ResNet152`` accept ``num_classes`` (reference ignores it,
    `pytorch_model.py:109-113`).
  * ``stem='imagenet'`` adds the 7x7/s2 conv + 3x3/s2 maxpool stem and an
    adaptive average pool so ResNet-50 runs at 224x224 (reference fails, F9).
"""
from __future__ import annotations

import torch.nn as nn
import torch.nn.functional as F


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, planes * self.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * self.expansion))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        return F.relu(out + self.shortcut(x))


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_planes, planes, stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * self.expansion, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.shortcut = nn.Sequential()
        if stride != 1 or in_planes != planes * self.expansion:
            self.shortcut = nn.Sequential(
                nn.Conv2d(in_planes, planes * self.expansion, 1, stride, bias=False),
                nn.BatchNorm2d(planes * self.expansion))

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        out = F.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return F.relu(out + self.shortcut(x))


class ResNet(nn.Module):
    def __init__(self, block, num_blocks, num_classes=10, stem='cifar', in_channels=3):
        super().__init__()
        self.in_planes = 64
        self.stem = stem
        if stem == 'cifar':
            self.conv1 = nn.Conv2d(in_channels, 64, 3, 1, 1, bias=False)
        elif stem == 'imagenet':
            self.conv1 = nn.Conv2d(in_channels, 64, 7, 2, 3, bias=False)
        else:
            raise ValueError(stem)
        self.bn1 = nn.BatchNorm2d(64)
        self.layer1 = self._make_layer(block, 64, num_blocks[0], 1)
        self.layer2 = self._make_layer(block, 128, num_blocks[1], 2)
        self.layer3 = self._make_layer(block, 256, num_blocks[2], 2)
        self.layer4 = self._make_layer(block, 512, num_blocks[3], 2)
        self.linear = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, num_blocks, stride):
        layers = []
        for s in [stride] + [1] * (num_blocks - 1):
            layers.append(block(self.in_planes, planes, s))
            self.in_planes = planes * block.expansion
        return nn.Sequential(*layers)

    def forward(self, x):
        out = F.relu(self.bn1(self.conv1(x)))
        if self.stem == 'imagenet':
            out = F.max_pool2d(out, 3, 2, 1)
        out = self.layer4(self.layer3(self.layer2(self.layer1(out))))
        if self.stem == 'imagenet':
            out = F.adaptive_avg_pool2d(out, 1)
        else:
            out = F.avg_pool2d(out, 4)
        return self.linear(out.flatten(1))


def ResNet18(num_classes=10, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes, **kw)


def ResNet34(num_classes=10, **kw):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes, **kw)


def ResNet50(num_classes=10, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, **kw)


def ResNet101(num_classes=10, **kw):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes, **kw)


def ResNet152(num_classes=10, **kw):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes, **kw)


def ResNet50_ImageNet(num_classes=1000):
    """ResNet-50 with the ImageNet stem for 224x224 (BASELINE config 5)."""
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes, stem='imagenet')
